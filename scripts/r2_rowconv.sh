# 64-channel 3x3 row kernel: numerics vs the implicit-GEMM tiles, then step A/B (DPE_ROWCONV=0/1) + profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "rowconv or conv_fwd or conv_dgrad" > gpurun_out/rc_tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/rc_tests.log | head -30; tail -30 gpurun_out/rc_tests.log; exit 1; }
tail -1 gpurun_out/rc_tests.log
for r in 1 2; do for v in 0 1; do
  DPE_ROWCONV=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/rc.log 2>&1 || exit 1
  echo "rowconv=$v $(tail -1 gpurun_out/rc.log | cut -c100-190)"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_rc -o run -- python bench.py --steps 6 --warmup 3 > gpurun_out/prof_rc.log 2>&1 || exit 1
