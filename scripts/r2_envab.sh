# re-measure older dispatch alternatives against the current default (alternating, bench.py 30 steps)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in "X=0" "DPE_WGRAD_DMA=2" "DPE_DMA_ALL=1" "DPE_WGRAD_HGEMM=0"; do
    env $v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/envab.log 2>&1 || exit 1
    echo "$v $(tail -1 gpurun_out/envab.log | cut -c100-190)"
  done
done
