#!/bin/bash
# On-load BN applies (igemm AXform): op numerics, model-level tests, then alternating A/B benches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/ax
timeout -k 10 300 python -u -m pytest tests/test_bnin_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/ax/bnin.log 2>&1 || { echo "BNIN TESTS FAILED"; tail -40 gpurun_out/ax/bnin.log; exit 1; }
tail -1 gpurun_out/ax/bnin.log
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py tests/test_model_parity_gpu.py tests/test_comm_gpu.py -x -q -s \
  --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/ax/models.log 2>&1 || { echo "MODEL TESTS FAILED"; tail -40 gpurun_out/ax/models.log; exit 1; }
tail -1 gpurun_out/ax/models.log
ARMS="${ARMS:-- DPE_AX_FWD=0,DPE_AX_BWD=0 DPE_AX_TILE=256}" MODEL=resnet50 ROUNDS=${ROUNDS:-2} bash scripts/ab_bench.sh
