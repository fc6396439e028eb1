#!/bin/bash
# BN3 Gram path: kernel tests, ResNet-50 on/off step test, then an on/off bench A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/gram
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_bn3_gram_gpu.py > gpurun_out/gram/tests.log 2>&1 || { echo "GRAM TESTS FAILED"; grep -E "PASSED|FAILED|Error|assert" gpurun_out/gram/tests.log | head -30; tail -50 gpurun_out/gram/tests.log; exit 1; }
grep -E "PASSED|FAILED|worst" gpurun_out/gram/tests.log | cut -c1-200
for arm in 0 1 0 1; do
  DPE_BN3_GRAM=$arm timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/gram/bench_$arm.log 2>&1 || { tail -20 gpurun_out/gram/bench_$arm.log; exit 1; }
  echo "gram=$arm $(tail -1 gpurun_out/gram/bench_$arm.log | cut -c1-110)"
done
