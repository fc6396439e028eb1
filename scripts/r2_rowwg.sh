# row-walking 3x3 weight grad: numerics, per-shape A/B, step A/B (DPE_ROW_WGRAD=0/1), one-step profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "row_wgrad or wgrad or rowconv" > gpurun_out/rw_tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/rw_tests.log | head -30; tail -30 gpurun_out/rw_tests.log; exit 1; }
tail -1 gpurun_out/rw_tests.log
timeout -k 10 200 python -u scripts/row_wgrad_ab.py > gpurun_out/rw_ab.log 2>&1 || { tail -20 gpurun_out/rw_ab.log; exit 1; }
cat gpurun_out/rw_ab.log
for r in 1 2; do for v in 0 1; do
  DPE_ROW_WGRAD=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/rw.log 2>&1 || exit 1
  echo "row_wgrad=$v $(tail -1 gpurun_out/rw.log | cut -c100-190)"
done; done
