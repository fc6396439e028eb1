set -o pipefail
# CE kernel-side mean: numerics tests, then the per-kernel hog factors through the production path
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_parity_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6b_tests.log 2>&1 || { tail -30 gpurun_out/r6b_tests.log; exit 1; }
tail -1 gpurun_out/r6b_tests.log
TRACE_ONLY=1 bash scripts/gpu_hog.sh 16 256 19968 140 0 > gpurun_out/hog_kernels.txt 2>&1; tail -60 gpurun_out/hog_kernels.txt
timeout -k 10 300 python scripts/bench_dgrad_bnb.py > gpurun_out/dgrad_bnb.txt 2>&1; cat gpurun_out/dgrad_bnb.txt
