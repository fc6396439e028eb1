# ping-pong prefetch in the row weight-grad kernels: numerics, per-kernel timings, bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "stem or row or resnet or bottleneck or chained" > gpurun_out/pp_tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/pp_tests.log | head -30; tail -30 gpurun_out/pp_tests.log; exit 1; }
tail -1 gpurun_out/pp_tests.log
timeout -k 10 200 python -u scripts/stem_wgrad_ab.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python -u scripts/row_wgrad_ab.py 2>&1 | grep -v amdgpu.ids
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/pp.log 2>&1 || exit 1
  echo "$(tail -1 gpurun_out/pp.log | cut -c100-190)"
done
