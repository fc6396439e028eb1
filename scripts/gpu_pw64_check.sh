#!/bin/bash
# K=64 pointwise data grad at 32 columns per wave: pw / conv / model tests, then A/B vs the WN=64 variant,
# then the world-2 rehearsal of the driver's multi-rank bench path
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/pw64
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pw64/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/pw64/tests.log; exit 1; }
tail -1 gpurun_out/pw64/tests.log
ARMS="- DPE_EXT_SO=$R/distributed_pytorch_example_amd/_C_pw64.so" MODEL=resnet50 ROUNDS=3 bash scripts/ab_bench.sh || exit 1
bash scripts/bench_world2_1gpu.sh
