#!/bin/bash
# Strided data grads: base vs the 8-row BN-backward epilogue batch (v_g8.so), then the ResNet-50 bench A/B.
set -o pipefail
for arm in base g8; do
  so=abso/base_C.so; [ $arm = g8 ] && so=distributed_pytorch_example_amd/v_g8.so
  echo "== $arm"
  DPE_EXT_SO=$so MODES=0 timeout -k 10 200 python -u scripts/bench_phase_dgrad.py || exit 1
done
for r in 1 2; do
  for arm in A B; do
    so=abso/base_C.so; [ $arm = B ] && so=distributed_pytorch_example_amd/v_g8.so
    DPE_EXT_SO=$so timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_$arm.log 2>&1 || { tail -5 gpurun_out/ab_$arm.log; exit 1; }
    echo "$arm $(grep '"metric"' gpurun_out/ab_$arm.log | python3 -c 'import json,sys; l=json.loads(sys.stdin.read()); print(l["value"], l["ms_per_step"])')"
  done
done
