#!/bin/bash
# BN-backward reduce blocks at >= 1024 channels: DPE_BNR_ROWS 64 (default) vs 16 vs 32, bench, alternating.
set -o pipefail
for r in 1 2; do
  for rows in 64 16 32; do
    DPE_BNR_ROWS=$rows timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bnr.log 2>&1 || { tail -5 gpurun_out/bnr.log; exit 1; }
    echo "rows=$rows $(grep '"metric"' gpurun_out/bnr.log | python3 -c 'import json,sys; l=json.loads(sys.stdin.read()); print(l["value"], l["ms_per_step"])')"
  done
done
for arm in base ns3; do
  so=distributed_pytorch_example_amd/_C.so; [ $arm = ns3 ] && so=distributed_pytorch_example_amd/v_ns3.so
  echo "== $arm"
  DPE_EXT_SO=$so MODES=0 timeout -k 10 200 python -u scripts/bench_phase_dgrad.py 2>&1 | grep -v amdgpu.ids || exit 1
done
