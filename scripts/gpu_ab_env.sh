#!/bin/bash
# Same-box A/B of an env toggle on the 1-GPU bench: bash scripts/gpu_ab_env.sh <model> <VAR=val (B arm)> [rounds]
# (A arm: the default environment).  Alternating processes; one JSON summary line per run.
set -o pipefail
mkdir -p gpurun_out/ab
M=${1:-resnet50}; B=$2; N=${3:-2}
for r in $(seq 1 $N); do
  for arm in A B; do
    if [ $arm = A ]; then timeout -k 10 200 python bench.py --model $M --steps 20 --warmup 5 > gpurun_out/ab/$arm.log 2>&1 || { tail -20 gpurun_out/ab/$arm.log; exit 1; }
    else timeout -k 10 200 env $B python bench.py --model $M --steps 20 --warmup 5 > gpurun_out/ab/$arm.log 2>&1 || { tail -20 gpurun_out/ab/$arm.log; exit 1; }; fi
    echo "$arm $(grep '"metric"' gpurun_out/ab/$arm.log | python3 -c 'import json,sys; l=json.loads(sys.stdin.read()); print(l["value"], l["ms_per_step"])')"
  done
done
