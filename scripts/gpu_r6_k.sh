#!/bin/bash
# Conv epilogue staging without the per-element bias / activation tests: numerics, per-shape benches and a
# same-box bench A/B against abso/base_C.so (the previous build).
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py 2>&1 | tail -2 || exit 1
for arm in base new; do
  so=abso/base_C.so; [ $arm = new ] && so=distributed_pytorch_example_amd/_C.so
  echo "== $arm"
  DPE_EXT_SO=$so MODES=0 timeout -k 10 200 python -u scripts/bench_phase_dgrad.py 2>&1 | grep -v amdgpu.ids || exit 1
  DPE_EXT_SO=$so timeout -k 10 200 python -u scripts/bench_dgrad_bnb.py 2>&1 | grep -v amdgpu.ids | head -3 || exit 1
done
for r in 1 2 3; do
  for arm in A B; do
    so=abso/base_C.so; [ $arm = B ] && so=distributed_pytorch_example_amd/_C.so
    DPE_EXT_SO=$so timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_$arm.log 2>&1 || { tail -5 gpurun_out/ab_$arm.log; exit 1; }
    echo "$arm $(grep '"metric"' gpurun_out/ab_$arm.log | python3 -c 'import json,sys; l=json.loads(sys.stdin.read()); print(l["value"], l["ms_per_step"])')"
  done
done
