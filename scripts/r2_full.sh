set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r2_gputest.log 2>&1; rc=$?; tail -3 gpurun_out/r2_gputest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/r2_gputest.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/r2_bench_r50.log 2>&1 && tail -1 gpurun_out/r2_bench_r50.log || exit 1
timeout -k 10 300 python bench.py --model gpt2 > gpurun_out/r2_bench_gpt2.log 2>&1 && tail -1 gpurun_out/r2_bench_gpt2.log || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_smoke.log 2>&1 && tail -1 gpurun_out/r2_smoke.log
