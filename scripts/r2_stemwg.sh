# row-walking stem weight grad: numerics, per-shape A/B, step A/B (DPE_STEM_WGRAD=0/1)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "stem or resnet" > gpurun_out/sw_tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/sw_tests.log | head -30; tail -30 gpurun_out/sw_tests.log; exit 1; }
tail -1 gpurun_out/sw_tests.log
timeout -k 10 200 python -u scripts/stem_wgrad_ab.py > gpurun_out/sw_ab.log 2>&1 || { tail -20 gpurun_out/sw_ab.log; exit 1; }
cat gpurun_out/sw_ab.log
for r in 1 2; do for v in 0 1; do
  DPE_STEM_WGRAD=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/sw.log 2>&1 || exit 1
  echo "stem_wgrad=$v $(tail -1 gpurun_out/sw.log | cut -c100-190)"
done; done
