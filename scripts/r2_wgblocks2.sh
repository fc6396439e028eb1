# register-staged 1x1 weight grads at 512 blocks + LDS-DMA im2col weight grads at 768 (default) vs both at 768
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad or conv or resnet or bottleneck" > gpurun_out/wb2_tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/wb2_tests.log | head -30; tail -30 gpurun_out/wb2_tests.log; exit 1; }
tail -1 gpurun_out/wb2_tests.log
for r in 1 2 3; do for v in 512 768; do
  DPE_WGRAD_BLOCKS=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/wb.log 2>&1 || exit 1
  echo "reg_wgrad_blocks=$v $(tail -1 gpurun_out/wb.log | cut -c100-190)"
done; done
