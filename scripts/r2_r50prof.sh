set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o run -- python bench.py --steps 8 --warmup 3 > gpurun_out/r2_prof_r50.log 2>&1 || exit 1
timeout -k 10 400 python scripts/bench_convs.py --batch 512 --reps 10 --miopen 0 > gpurun_out/r2_convs.txt 2>&1; tail -30 gpurun_out/r2_convs.txt
