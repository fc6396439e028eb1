#!/bin/bash
# rocprofv3 kernel-trace/stats of bench.py (and optionally the stock arm); summaries in gpurun_out/prof*
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o ours -- python3 $R/bench.py --steps 5 --warmup 2 ${BENCH_ARGS} > $R/gpurun_out/prof_ours.log 2>&1 || { echo "PROF OURS FAILED"; tail -20 $R/gpurun_out/prof_ours.log; exit 1; }
tail -1 $R/gpurun_out/prof_ours.log
if [ "${STOCK:-0}" = "1" ]; then
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o stock -- python3 $R/scripts/bench_stock.py --steps 5 --warmup 3 > $R/gpurun_out/prof_stock.log 2>&1 || { echo "PROF STOCK FAILED"; tail -20 $R/gpurun_out/prof_stock.log; exit 1; }
tail -1 $R/gpurun_out/prof_stock.log
fi
find $R/gpurun_out/prof -name "*stats*"
