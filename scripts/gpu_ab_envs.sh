#!/bin/bash
# Tests, then conv microbench + bench.py under a list of env settings ("A=1,B=2" per arm; "-" = none).
# usage: ARMS="DPE_DMA_TILE=128,DPE_WGRAD_WIDE=0 -" bash scripts/gpu_ab_envs.sh
set -o pipefail
mkdir -p gpurun_out
[ "${SKIPTEST:-0}" = "1" ] || { timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -m gpu --timeout 120 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/kt.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/kt.log; exit 1; }; tail -1 gpurun_out/kt.log; }
i=0
for arm in $ARMS; do
  i=$((i+1)); envs=$(echo "$arm" | tr ',' ' '); [ "$arm" = "-" ] && envs=""
  if [ "${CONVS:-1}" = "1" ]; then
    env $envs timeout -k 10 300 python scripts/bench_convs.py --batch ${BATCH:-512} --reps 10 --miopen 0 > gpurun_out/convs_arm$i.txt 2>&1 || { echo "CONVS $arm FAILED"; tail -20 gpurun_out/convs_arm$i.txt; exit 1; }
    echo "== convs [$arm]: $(grep '^ours' gpurun_out/convs_arm$i.txt)"
  fi
  if [ "${BENCH:-1}" = "1" ]; then
    env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS} > gpurun_out/bench_arm$i.log 2>&1 || { echo "BENCH $arm FAILED"; tail -20 gpurun_out/bench_arm$i.log; exit 1; }
    echo "== bench [$arm]: $(tail -1 gpurun_out/bench_arm$i.log | cut -c100-200)"
  fi
done
