set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pool_test.log 2>&1; rc=$?; tail -1 gpurun_out/pool_test.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED|^E " gpurun_out/pool_test.log | head; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_r50c -o run -- python bench.py --steps 8 --warmup 3 > gpurun_out/prof_r50c.log 2>&1 || exit 1
python scripts/prof_steady.py $(find gpurun_out/prof_r50c -name "*.db" | head -1) 2 sgd_kernel 60 > gpurun_out/r50_steady_c.txt
head -1 gpurun_out/r50_steady_c.txt; grep -i pool gpurun_out/r50_steady_c.txt
timeout -k 10 200 python bench.py > gpurun_out/r2_bench_r50.log 2>&1 && tail -1 gpurun_out/r2_bench_r50.log | cut -c1-150
