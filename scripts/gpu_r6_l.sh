#!/bin/bash
# 1x1 forwards with BN statistics at depth 512 (>= 256 outputs) on the persistent GEMM: DPE_HG_BNF_MINK 1024 vs 512.
set -o pipefail
for r in 1 2 3; do
  for k in 1024 512; do
    DPE_HG_BNF_MINK=$k timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bnf.log 2>&1 || { tail -5 gpurun_out/bnf.log; exit 1; }
    echo "mink=$k $(grep '"metric"' gpurun_out/bnf.log | python3 -c 'import json,sys; l=json.loads(sys.stdin.read()); print(l["value"], l["ms_per_step"])')"
  done
done
DPE_HG_BNF_MINK=512 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_models_gpu.py tests/test_model_parity_gpu.py 2>&1 | tail -2
