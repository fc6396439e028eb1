#!/bin/bash
# LayerNorm backward, whole-row lean form (all row operands loaded first, clamped tail lanes, compile-time
# output form): numerics, then GPT-2 bench DPE_LN_BWD_LEAN=0 vs 1 alternating.
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "layernorm or ln_ or norm" \
  tests/test_models_gpu.py tests/test_model_parity_gpu.py 2>&1 | tail -2 || exit 1
for r in 1 2 3; do
  for v in 0 1; do
    DPE_LN_BWD_LEAN=$v timeout -k 10 200 python bench.py --model gpt2 --steps 20 --warmup 5 > gpurun_out/lnl.log 2>&1 || { tail -5 gpurun_out/lnl.log; exit 1; }
    echo "lean=$v $(grep '"metric"' gpurun_out/lnl.log | python3 -c 'import json,sys; l=json.loads(sys.stdin.read()); print(l["value"], l["ms_per_step"])')"
  done
done
