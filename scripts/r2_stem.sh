# stem kernel: numerics vs the implicit-GEMM tile, model tests, then step A/B (DPE_STEM=0/1) + profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "stem or conv_fwd" > gpurun_out/stem_tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/stem_tests.log | head -30; tail -30 gpurun_out/stem_tests.log; exit 1; }
tail -1 gpurun_out/stem_tests.log
for r in 1 2; do for v in 0 1; do
  DPE_STEM=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/stem.log 2>&1 || exit 1
  echo "stem=$v $(tail -1 gpurun_out/stem.log | cut -c100-190)"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_stemk -o run -- python bench.py --steps 6 --warmup 3 > gpurun_out/prof_stemk.log 2>&1 || exit 1
