# A/B of the 1x1 conv weight grads: implicit-GEMM atomic path vs persistent hgemm + split-K slabs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv or wgrad" > gpurun_out/wg_tests.log 2>&1 || { tail -30 gpurun_out/wg_tests.log; exit 1; }
tail -2 gpurun_out/wg_tests.log
for v in 0 1; do
  DPE_WGRAD_HGEMM=$v timeout -k 10 240 python -u scripts/bench_convs.py --batch 512 --miopen 0 --reps 10 > gpurun_out/wg_convs_$v.log 2>&1 || exit 1
  grep wgrad gpurun_out/wg_convs_$v.log
done
for v in 0 1 0 1; do
  DPE_WGRAD_HGEMM=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/wg_bench_$v.log 2>&1 || exit 1
  echo "hgemm=$v $(tail -1 gpurun_out/wg_bench_$v.log)"
done
