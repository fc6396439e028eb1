# pw_stream K=256 data grad with hoisted epilogue operand loads: numerics, bench, kernel times
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_ddp_rccl_world2_gpu.py -x -q --timeout 150 --timeout-method thread -k "pw or resnet or bottleneck or chained or world2" > gpurun_out/ph_tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/ph_tests.log | head -30; tail -30 gpurun_out/ph_tests.log; exit 1; }
tail -1 gpurun_out/ph_tests.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/ph.log 2>&1 || exit 1
  echo "r50 $(tail -1 gpurun_out/ph.log | cut -c100-175)"
done
rm -rf gpurun_out/prof_ph
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_ph -o run -- python bench.py --steps 8 --warmup 3 > gpurun_out/prof_ph.log 2>&1 || exit 1
python scripts/prof_steady.py $(find gpurun_out/prof_ph -name "*.db" | head -1) 2 sgd_kernel 60 > gpurun_out/r50_steady_ph.txt
grep -E "wall|pw_stream" gpurun_out/r50_steady_ph.txt
rm -rf gpurun_out/prof_ph
