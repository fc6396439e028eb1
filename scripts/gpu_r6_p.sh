#!/bin/bash
# GPT-2 same-box A/B of the current build against abso/base_C.so (previous build), with the LayerNorm tests.
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "layernorm" 2>&1 | tail -1 || exit 1
for r in 1 2 3; do
  for arm in A B; do
    so=abso/base_C.so; [ $arm = B ] && so=distributed_pytorch_example_amd/_C.so
    DPE_EXT_SO=$so timeout -k 10 200 python bench.py --model gpt2 --steps 20 --warmup 5 > gpurun_out/ab_$arm.log 2>&1 || { tail -5 gpurun_out/ab_$arm.log; exit 1; }
    echo "$arm $(grep '"metric"' gpurun_out/ab_$arm.log | python3 -c 'import json,sys; l=json.loads(sys.stdin.read()); print(l["value"], l["ms_per_step"])')"
  done
done
