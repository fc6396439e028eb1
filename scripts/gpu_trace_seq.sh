#!/bin/bash
# One ResNet-50 steady step, kernel by kernel (env passed through), into gpurun_out/seq/$TAG.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/seq
cd /tmp && export TMPDIR=/tmp
TAG=${TAG:-run}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/seq/tr_$TAG -o run -- python3 $R/bench.py --steps 5 --warmup 3 ${BENCH_ARGS} > $R/gpurun_out/seq/$TAG.log 2>&1 || { tail -20 $R/gpurun_out/seq/$TAG.log; exit 1; }
f=$(find $R/gpurun_out/seq/tr_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/scripts/prof_sequence.py $f 4 ${MARK:-sgd_kernel} > $R/gpurun_out/seq/$TAG.txt
python3 $R/scripts/prof_steady.py $f 3 ${MARK:-sgd_kernel} 45 > $R/gpurun_out/seq/${TAG}_steady.txt
rm -rf $R/gpurun_out/seq/tr_$TAG
head -3 $R/gpurun_out/seq/${TAG}_steady.txt
