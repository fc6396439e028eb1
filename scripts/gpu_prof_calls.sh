#!/bin/bash
# One kernel trace of bench.py; per-call durations of the kernels matching each FILTERS word (one steady step)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/calls
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/calls/tr -o run -- python3 $R/bench.py --steps 6 --warmup 3 ${BENCH_ARGS} > $R/gpurun_out/calls/trace.log 2>&1 || { echo "TRACE FAILED"; tail -20 $R/gpurun_out/calls/trace.log; exit 1; }
f=$(find $R/gpurun_out/calls/tr -name "*kernel_trace.csv" | head -1)
for w in ${FILTERS}; do python3 $R/scripts/prof_calls.py $f "$w" ${MARK:-sgd_kernel} 4 > $R/gpurun_out/calls/$w.txt; done
head -3 $f | cut -c1-400 > $R/gpurun_out/calls/header.txt
rm -rf $R/gpurun_out/calls/tr
