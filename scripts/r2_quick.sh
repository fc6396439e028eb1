set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hgemm_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/q_test.log 2>&1; rc=$?; tail -2 gpurun_out/q_test.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --model gpt2 > gpurun_out/r2_bench_gpt2.log 2>&1 && tail -1 gpurun_out/r2_bench_gpt2.log | cut -c1-200
