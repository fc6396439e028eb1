# split-K block target of the implicit-GEMM weight grads (DPE_WGRAD_BLOCKS), ResNet-50 step, alternating
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in 768 640 704 832 896; do
    DPE_WGRAD_BLOCKS=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/wb.log 2>&1 || exit 1
    echo "wgrad_blocks=$v $(tail -1 gpurun_out/wb.log | cut -c100-190)"
  done
done
