# DPE_DMA_ALL A/B (every forward-form conv role on the LDS-DMA kernel), alternating, 40 steps
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in 0 1; do
    DPE_DMA_ALL=$v timeout -k 10 300 python -u bench.py --steps 40 --warmup 10 > gpurun_out/da.log 2>&1 || exit 1
    echo "dma_all=$v $(tail -1 gpurun_out/da.log | cut -c100-190)"
  done
done
