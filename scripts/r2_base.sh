set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_gputest.log 2>&1 && tail -2 gpurun_out/r2_gputest.log &&
timeout -k 10 300 python bench.py > gpurun_out/r2_bench_r50.log 2>&1 && tail -1 gpurun_out/r2_bench_r50.log &&
timeout -k 10 300 python bench.py --model gpt2 > gpurun_out/r2_bench_gpt2.log 2>&1 && tail -1 gpurun_out/r2_bench_gpt2.log &&
timeout -k 10 200 python scripts/bench_gemm_shapes.py square > gpurun_out/r2_gemm_square.log 2>&1 && cat gpurun_out/r2_gemm_square.log
