set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_r50b -o run -- python bench.py --steps 8 --warmup 3 > gpurun_out/prof_r50b.log 2>&1 || exit 1
python scripts/prof_steady.py $(find gpurun_out/prof_r50b -name "*.db" | head -1) 2 sgd_kernel 45 > gpurun_out/r50_steady_b.txt
head -30 gpurun_out/r50_steady_b.txt
