# layer-1 a1 never materialised (BN1+ReLU on load in the row kernels): numerics, then step A/B (DPE_ROW_BNIN=0/1)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "row or bottleneck or chained or resnet or wgrad" > gpurun_out/rb_tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/rb_tests.log | head -30; tail -30 gpurun_out/rb_tests.log; exit 1; }
tail -1 gpurun_out/rb_tests.log
for r in 1 2; do for v in 0 1; do
  DPE_ROW_BNIN=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/rb.log 2>&1 || exit 1
  echo "row_bnin=$v $(tail -1 gpurun_out/rb.log | cut -c100-190)"
done; done
