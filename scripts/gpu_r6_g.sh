#!/bin/bash
# Stem max-pool key-max kernel: numerics tests, then a same-box bench A/B against abso/base_C.so and a
# kernel-trace of both arms' steady steps.
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "maxpool or stem or bn or pool or resnet" 2>&1 | tail -3 || exit 1
for r in 1 2 3; do
  for arm in A B; do
    so=abso/base_C.so; [ $arm = B ] && so=distributed_pytorch_example_amd/_C.so
    DPE_EXT_SO=$so timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_$arm.log 2>&1 || { tail -5 gpurun_out/ab_$arm.log; exit 1; }
    echo "$arm $(grep '"metric"' gpurun_out/ab_$arm.log | python3 -c 'import json,sys; l=json.loads(sys.stdin.read()); print(l["value"], l["ms_per_step"])')"
  done
done
