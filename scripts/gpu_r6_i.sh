#!/bin/bash
# Strided data grads in one grouped launch: numerics, per-shape bench (grouped vs per parity), bench A/B.
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "phase_group or dgrad or strided" 2>&1 | tail -3 || exit 1
for grp in 1 0; do
  echo "== DPE_PHASE_GROUP=$grp"
  DPE_PHASE_GROUP=$grp MODES=0 timeout -k 10 200 python -u scripts/bench_phase_dgrad.py 2>&1 | grep -v amdgpu.ids || exit 1
done
for r in 1 2 3; do
  for grp in 0 1; do
    DPE_PHASE_GROUP=$grp timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/pg.log 2>&1 || { tail -5 gpurun_out/pg.log; exit 1; }
    echo "group=$grp $(grep '"metric"' gpurun_out/pg.log | python3 -c 'import json,sys; l=json.loads(sys.stdin.read()); print(l["value"], l["ms_per_step"])')"
  done
done
