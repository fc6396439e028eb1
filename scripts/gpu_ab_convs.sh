#!/bin/bash
# A/B of an env toggle on the conv microbench (+ optionally bench.py): tests -> convs per value -> bench per value.
# usage: TOGGLE=DPE_DMA_TILE VALS="128 256x128" BENCH=1 bash scripts/gpu_ab_convs.sh
set -o pipefail
mkdir -p gpurun_out
T=${TOGGLE:-DPE_IGEMM_DMA}
VALS=${VALS:-"0 1"}
[ "${SKIPTEST:-0}" = "1" ] || timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -m gpu --timeout 120 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/kt.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/kt.log; exit 1; }
[ "${SKIPTEST:-0}" = "1" ] || tail -2 gpurun_out/kt.log
[ "${CONVS:-1}" = "1" ] && for v in $VALS; do
  env $T=$v timeout -k 10 300 python scripts/bench_convs.py --batch ${BATCH:-512} --reps 10 --miopen 0 > gpurun_out/convs_$v.txt 2>&1 || { echo "CONVS $v FAILED"; tail -20 gpurun_out/convs_$v.txt; exit 1; }
  echo "== $T=$v"; tail -3 gpurun_out/convs_$v.txt | head -1
done
if [ "${BENCH:-1}" = "1" ]; then
for v in $VALS; do
  env $T=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_$v.log 2>&1 || { echo "BENCH $v FAILED"; tail -20 gpurun_out/bench_$v.log; exit 1; }
  echo "== bench $T=$v"; tail -1 gpurun_out/bench_$v.log | cut -c1-200
done
fi
