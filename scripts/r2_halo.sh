set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "halo or conv_fwd or conv_dgrad" > gpurun_out/halo_tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/halo_tests.log | head -30; tail -30 gpurun_out/halo_tests.log; exit 1; }
tail -1 gpurun_out/halo_tests.log
timeout -k 10 200 python -u scripts/halo_ab.py > gpurun_out/halo_ab.log 2>&1 || { cat gpurun_out/halo_ab.log; exit 1; }
cat gpurun_out/halo_ab.log
for v in 0 1 0 1; do
  DPE_CONV3_HALO=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/halo_bench.log 2>&1 || exit 1
  echo "halo=$v $(tail -1 gpurun_out/halo_bench.log | cut -c100-190)"
done
