#!/bin/bash
# Alternating A/B of bench.py under env settings: ROUNDS rounds x every arm ("A=1,B=2" per arm,
# "-" = none), one process per run, so drift between boxes / DVFS states hits every arm alike.
# usage: ARMS="DPE_FINALIZE_STREAM=1 -" MODEL=gpt2 ROUNDS=3 bash scripts/ab_bench.sh
set -o pipefail
mkdir -p gpurun_out/ab
ROUNDS=${ROUNDS:-3}
for r in $(seq 1 $ROUNDS); do
  i=0
  for arm in $ARMS; do
    i=$((i+1)); envs=$(echo "$arm" | tr ',' ' '); [ "$arm" = "-" ] && envs=""
    log=gpurun_out/ab/${MODEL:-resnet50}_arm${i}_r$r.log
    env $envs timeout -k 10 240 python bench.py --model ${MODEL:-resnet50} --steps ${STEPS:-15} --warmup ${WARMUP:-4} ${BENCH_ARGS} > $log 2>&1 || { echo "BENCH [$arm] FAILED"; tail -20 $log; exit 1; }
    echo "${MODEL:-resnet50} round $r [$arm] $(tail -1 $log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/step", round(d["value"]), d["unit"])')"
  done
done
