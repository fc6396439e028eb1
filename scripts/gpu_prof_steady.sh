#!/bin/bash
# Steady-state kernel breakdown of bench.py (rocprofv3 kernel trace) + per-shape conv table.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
MARK=${MARK:-sgd_kernel}
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace -o run -- python3 $R/bench.py --steps 8 --warmup 3 ${BENCH_ARGS} > $R/gpurun_out/trace.log 2>&1 || { echo "TRACE FAILED"; tail -20 $R/gpurun_out/trace.log; exit 1; }
tail -1 $R/gpurun_out/trace.log
f=$(find $R/gpurun_out/trace -name "*kernel_trace.csv" | head -1)
python3 $R/scripts/prof_steady.py $f 4 $MARK ${TOP:-70} > $R/gpurun_out/steady.txt && cat $R/gpurun_out/steady.txt
rm -f $f
if [ "${CONVS:-0}" = "1" ]; then
cd $R && timeout -k 10 400 python3 scripts/bench_convs.py --reps 10 > gpurun_out/convs.txt 2>&1 || { echo "CONVS FAILED"; tail -20 gpurun_out/convs.txt; exit 1; }
tail -3 gpurun_out/convs.txt
fi
