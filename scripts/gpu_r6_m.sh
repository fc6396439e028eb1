#!/bin/bash
# BN apply / backward-apply without run-time-tested loads and stores (lean kernels): numerics, then the
# ResNet-50 bench with DPE_BN_BWD_LEAN=0 (generic kernels) vs 1, alternating.
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py \
  tests/test_model_parity_gpu.py tests/test_bn3_gram_gpu.py 2>&1 | tail -2 || exit 1
for r in 1 2 3; do
  for v in 0 1; do
    DPE_BN_BWD_LEAN=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/lean.log 2>&1 || { tail -5 gpurun_out/lean.log; exit 1; }
    echo "lean=$v $(grep '"metric"' gpurun_out/lean.log | python3 -c 'import json,sys; l=json.loads(sys.stdin.read()); print(l["value"], l["ms_per_step"])')"
  done
done
