# hgemm planner K-split cap (DPE_HGEMM_SPLIT_CAP, default 128): ResNet-50 and GPT-2 steps, alternating
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in 128 8 16 32 64; do
    DPE_HGEMM_SPLIT_CAP=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/sc.log 2>&1 || exit 1
    echo "r50 split_cap=$v $(tail -1 gpurun_out/sc.log | cut -c100-175)"
  done
  for v in 128 8 16 32 64; do
    DPE_HGEMM_SPLIT_CAP=$v timeout -k 10 300 python -u bench.py --model gpt2 --steps 30 --warmup 5 > gpurun_out/sc.log 2>&1 || exit 1
    echo "gpt2 split_cap=$v $(tail -1 gpurun_out/sc.log | cut -c60-160)"
  done
done
