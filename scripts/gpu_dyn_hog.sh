#!/bin/bash
# RCCL-sized hogs (VALU-busy and idle) resident during backward: dynamic vs static GEMM schedule,
# with and without the CU budget.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/dyn
H="--threads 256 --lds 19968 --vgprs 136"
for m in gpt2 resnet50; do
  for sl in 0 1; do
    for d in 1 0; do
      f=gpurun_out/dyn/hog_${m}_s${sl}_d$d.jsonl
      DPE_HGEMM_DYNAMIC=$d timeout -k 10 300 python3 scripts/hog_probe.py --model $m $H --sleepy $sl --modes 0:0 16:0 16:16 > $f 2>&1 || { tail -20 $f; exit 1; }
      echo "model=$m sleepy=$sl dynamic=$d"; grep '^{' $f
    done
  done
done
