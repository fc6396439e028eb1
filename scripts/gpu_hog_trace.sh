#!/bin/bash
# Per-kernel trace of ResNet-50 with 16 RCCL-sized VALU-bound hogs + CU budget 16 vs no hogs (ENV: extra environment)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/hogtr
cd /tmp && export TMPDIR=/tmp
for m in 0:0 16:16; do
  tag=${m/:/_}
  env ${ENV} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/hogtr/t$tag -o run -- python3 $R/scripts/hog_probe.py --model resnet50 --threads 256 --lds 19968 --vgprs 140 --sleepy 0 --modes $m --rounds 1 --steps 5 > $R/gpurun_out/hogtr/t$tag.log 2>&1 || { tail -20 $R/gpurun_out/hogtr/t$tag.log; exit 1; }
done
f0=$(find $R/gpurun_out/hogtr/t0_0 -name "*kernel_trace.csv" | head -1)
f1=$(find $R/gpurun_out/hogtr/t16_16 -name "*kernel_trace.csv" | head -1)
python3 $R/scripts/prof_compare.py $f0 $f1 sgd_kernel 5 40
rm -f $f0 $f1
