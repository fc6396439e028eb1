#!/bin/bash
# Steady kernel summary AND one steady step in launch order (per-layer attribution) from one kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/seq
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/seq/tr -o run -- python3 $R/bench.py --steps 8 --warmup 3 ${BENCH_ARGS} > $R/gpurun_out/seq/trace.log 2>&1 || { echo "TRACE FAILED"; tail -20 $R/gpurun_out/seq/trace.log; exit 1; }
tail -1 $R/gpurun_out/seq/trace.log | cut -c1-200
f=$(find $R/gpurun_out/seq/tr -name "*kernel_trace.csv" | head -1)
python3 $R/scripts/prof_steady.py $f 4 ${MARK:-sgd_kernel} ${TOP:-80} > $R/gpurun_out/seq/steady.txt && head -3 $R/gpurun_out/seq/steady.txt
python3 $R/scripts/prof_sequence.py $f 4 ${MARK:-sgd_kernel} > $R/gpurun_out/seq/sequence.txt
rm -rf $R/gpurun_out/seq/tr
