#!/bin/bash
# One GPU session: kernel tests -> smoke -> our bench -> stock baseline. Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/kt.log 2>&1 || { echo "KERNEL TESTS FAILED"; tail -30 gpurun_out/kt.log; exit 1; }
tail -2 gpurun_out/kt.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --steps ${STEPS:-10} --warmup 3 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
if [ "${STOCK:-1}" = "1" ]; then
timeout -k 10 600 python scripts/bench_stock.py --steps 10 --warmup 5 > gpurun_out/stock.log 2>&1 || { echo "STOCK FAILED"; tail -20 gpurun_out/stock.log; exit 1; }
tail -1 gpurun_out/stock.log
fi
