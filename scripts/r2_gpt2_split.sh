# GPT-2 step: hgemm planner split cap 8 (before) vs 128 (one round of slots for few-tile GEMMs)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do for cap in 8 128; do
  DPE_HGEMM_SPLIT_CAP=$cap timeout -k 10 300 python -u bench.py --model gpt2 --steps 30 --warmup 10 > gpurun_out/g2s.log 2>&1 || exit 1
  echo "cap=$cap $(tail -1 gpurun_out/g2s.log | cut -c1-160)"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_gpt2c -o run -- python bench.py --model gpt2 --steps 8 --warmup 3 > gpurun_out/prof_gpt2c.log 2>&1 || exit 1
