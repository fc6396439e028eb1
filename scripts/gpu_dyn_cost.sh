#!/bin/bash
# Per-kernel cost of the CU-budget variants alone (reserve 16, no foreign workgroups) vs no budget.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/dyncost
cd /tmp && export TMPDIR=/tmp
for m in 0:0 0:16; do
  tag=${m/:/_}
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/dyncost/t$tag -o run -- python3 $R/scripts/hog_probe.py --model resnet50 --modes $m --rounds 1 --steps 5 > $R/gpurun_out/dyncost/t$tag.log 2>&1 || { tail -20 $R/gpurun_out/dyncost/t$tag.log; exit 1; }
done
f0=$(find $R/gpurun_out/dyncost/t0_0 -name "*kernel_trace.csv" | head -1)
f1=$(find $R/gpurun_out/dyncost/t0_16 -name "*kernel_trace.csv" | head -1)
python3 $R/scripts/prof_compare.py $f0 $f1 sgd_kernel 5 30
rm -f $f0 $f1
