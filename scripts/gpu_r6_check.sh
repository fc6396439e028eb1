set -o pipefail
# round-6 check: full GPU suite, both benches, world-8 one-GPU rehearsal of the bench (measured CU budget)
bash scripts/gpu_tests_bench.sh &&
timeout -k 10 300 python bench.py --model gpt2 --steps 10 --warmup 3 > gpurun_out/bench_gpt2.log 2>&1 && tail -1 gpurun_out/bench_gpt2.log | cut -c1-300 &&
bash scripts/world_1gpu.sh 8 resnet50 32 > gpurun_out/w8_rehearsal.txt 2>&1; tail -30 gpurun_out/w8_rehearsal.txt
