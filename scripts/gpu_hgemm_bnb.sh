#!/bin/bash
# 1x1 data grads (K >= 1024) on the persistent GEMM with the BN-backward epilogue: tests, then step A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/bnb
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_hgemm_gpu.py tests/test_models_gpu.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/bnb/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/bnb/tests.log; exit 1; }
tail -1 gpurun_out/bnb/tests.log
ARMS="- DPE_HGEMM_DGRAD=0" MODEL=resnet50 ROUNDS=3 bash scripts/ab_bench.sh
