set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad" > gpurun_out/wg_tests.log 2>&1 || { tail -30 gpurun_out/wg_tests.log; exit 1; }
tail -2 gpurun_out/wg_tests.log
timeout -k 10 200 python -u scripts/wg_grads.py 64 > gpurun_out/wg_grads.log 2>&1 || { cat gpurun_out/wg_grads.log; exit 1; }
cat gpurun_out/wg_grads.log
for v in 0 1 0 1; do
  DPE_WGRAD_HGEMM=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/wg_bench_$v.log 2>&1 || exit 1
  echo "hgemm=$v $(tail -1 gpurun_out/wg_bench_$v.log | cut -c1-200)"
done
