# LDS-DMA forward-conv tile choice (DPE_DMA_TILE: auto / 128 / 256x128 / 256x256), ResNet-50 step, alternating
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in auto 128 256x128 256x256; do
    DPE_DMA_TILE=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/dt.log 2>&1 || exit 1
    echo "dma_tile=$v $(tail -1 gpurun_out/dt.log | cut -c100-175)"
  done
done
