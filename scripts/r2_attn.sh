set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/attn_test.log 2>&1; rc=$?; tail -1 gpurun_out/attn_test.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 120 python scripts/bench_attn.py || exit 1
  DPE_EXT_SO=ab_so/_C_old.so timeout -k 10 120 python scripts/bench_attn.py || exit 1
done
