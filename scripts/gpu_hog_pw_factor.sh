#!/bin/bash
# same-box A/B of DPE_PW_DYN_FACTOR under the worst-case hog probe (ResNet-50, 16 VALU-bound RCCL-sized hogs, budget 16)
set -o pipefail
mkdir -p gpurun_out/hogab
for f in ${FACTORS:-3 8 3 8}; do
  DPE_PW_DYN_FACTOR=$f timeout -k 10 240 python3 scripts/hog_probe.py --model resnet50 --threads 256 --lds 19968 --vgprs 140 --sleepy 0 --modes 0:0 16:16 0:16 --rounds 1 --steps 6 > gpurun_out/hogab/f$f.log 2>&1 || { tail -20 gpurun_out/hogab/f$f.log; exit 1; }
  echo "factor $f: $(grep ms_step_median gpurun_out/hogab/f$f.log | python3 -c 'import sys,json; print([(json.loads(l)["hogs"],json.loads(l)["reserve"],json.loads(l)["ms_step_median"]) for l in sys.stdin if l.startswith("{")])')"
done
