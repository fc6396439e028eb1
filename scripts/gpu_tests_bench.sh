set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread > gpurun_out/kt_all.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/kt_all.log; exit 1; }
tail -1 gpurun_out/kt_all.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-230
