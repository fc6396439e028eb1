# steady-state kernel breakdowns of the ResNet-50 and GPT-2 benches (rocprofv3 kernel trace)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_r50c gpurun_out/prof_g2c
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_r50c -o run -- python bench.py --steps 8 --warmup 3 > gpurun_out/prof_r50c.log 2>&1 || exit 1
python scripts/prof_steady.py $(find gpurun_out/prof_r50c -name "*.db" | head -1) 2 sgd_kernel 60 > gpurun_out/r50_steady_c.txt
head -45 gpurun_out/r50_steady_c.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_g2c -o run -- python bench.py --model gpt2 --steps 8 --warmup 3 > gpurun_out/prof_g2c.log 2>&1 || exit 1
python scripts/prof_steady.py $(find gpurun_out/prof_g2c -name "*.db" | head -1) 2 adam_kernel 40 > gpurun_out/g2_steady_c.txt
head -30 gpurun_out/g2_steady_c.txt
rm -rf gpurun_out/prof_r50c gpurun_out/prof_g2c
