set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread > gpurun_out/kt_all.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/kt_all.log; exit 1; }
tail -1 gpurun_out/kt_all.log
for g in 0 1; do
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --graph $g > gpurun_out/bench_g$g.log 2>&1 || { echo "BENCH g$g FAILED"; tail -20 gpurun_out/bench_g$g.log; exit 1; }
echo "graph=$g"; tail -1 gpurun_out/bench_g$g.log | cut -c1-230
done
