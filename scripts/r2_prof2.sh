set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_r50 -o run -- python bench.py --steps 8 --warmup 3 > gpurun_out/prof_r50.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_gpt2 -o run -- python bench.py --model gpt2 --steps 8 --warmup 3 > gpurun_out/prof_gpt2.log 2>&1 || exit 1
python scripts/prof_steady.py $(find gpurun_out/prof_r50 -name "*.db" | head -1) 2 sgd_kernel 45 > gpurun_out/r50_steady.txt
python scripts/prof_steady.py $(find gpurun_out/prof_gpt2 -name "*.db" | head -1) 2 adam_kernel 40 > gpurun_out/gpt2_steady.txt
head -3 gpurun_out/r50_steady.txt; head -3 gpurun_out/gpt2_steady.txt
