set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r2_gputest.log 2>&1; rc=$?; tail -1 gpurun_out/r2_gputest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/r2_gputest.log | head -20; exit $rc; fi
for i in 1 2; do
timeout -k 10 300 python bench.py > gpurun_out/r2_bench_r50.log 2>&1 && tail -1 gpurun_out/r2_bench_r50.log | cut -c1-160 || exit 1
done
timeout -k 10 200 python scripts/bench_bn.py > gpurun_out/r2_bench_bn.txt 2>&1 && cat gpurun_out/r2_bench_bn.txt
