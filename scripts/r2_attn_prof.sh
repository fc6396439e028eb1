set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_attn -o run -- python scripts/bench_attn.py --reps 20 > gpurun_out/attn_prof.log 2>&1 || exit 1
f=$(find gpurun_out/prof_attn -name "*kernel_stats.csv" | head -1); cat "$f" | cut -d, -f1-8 | head -12
