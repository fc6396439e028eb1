#!/bin/bash
# Attention forward A/B: the kernel tests on each build, then bench_attn.py alternating builds
# (one process per run).  usage: SOS="a.so b.so" ROUNDS=3 bash scripts/gpu_attn_ab.sh
set -o pipefail
mkdir -p gpurun_out
P=distributed_pytorch_example_amd
for so in ${SOS}; do
  DPE_EXT_SO=$P/$so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_kernels_gpu.py -k attention > gpurun_out/attn_test_$so.log 2>&1 || { echo "TEST $so FAILED"; tail -30 gpurun_out/attn_test_$so.log; exit 1; }
  echo "tests $so: $(tail -1 gpurun_out/attn_test_$so.log)"
done
for r in $(seq 1 ${ROUNDS:-3}); do
  for so in ${SOS}; do
    DPE_EXT_SO=$P/$so timeout -k 10 120 python scripts/bench_attn.py --reps 50 || exit 1
  done
done
