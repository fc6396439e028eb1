#!/bin/bash
# Step-time table of the CU co-residency probe (profiles/cu_hog_probe_*): both models, whole-backward and windowed
# (W = 8 bucket windows at 300 GB/s) residency of 16 RCCL-sized VALU-bound hogs, modes 0:0 16:0 16:16 0:16.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/hogtab
cd $R
for w in 0 300; do
  for m in resnet50 gpt2; do
    timeout -k 10 300 python3 scripts/hog_probe.py --model $m --threads 256 --lds 19968 --vgprs 140 --sleepy 0 --windowed $w \
      --modes 0:0 16:0 16:16 0:16 > gpurun_out/hogtab/${m}_w$w.jsonl 2>&1 || { tail -20 gpurun_out/hogtab/${m}_w$w.jsonl; exit 1; }
    echo "## ${m}_w$w"; grep '^{' gpurun_out/hogtab/${m}_w$w.jsonl
  done
done
