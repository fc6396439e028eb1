#!/bin/bash
# inline-asm DMA + buffer-store by-products: conv / bnin numerics, microbench, then step A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/ax2
timeout -k 10 400 python -u -m pytest tests/test_bnin_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/ax2/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/ax2/tests.log; exit 1; }
tail -1 gpurun_out/ax2/tests.log
timeout -k 10 200 python -u scripts/bench_bnin.py > gpurun_out/ax2/bnin.jsonl 2>&1 || { tail -20 gpurun_out/ax2/bnin.jsonl; exit 1; }
grep op gpurun_out/ax2/bnin.jsonl
ARMS="- DPE_AX_FWD=0,DPE_AX_BWD=0 DPE_EXT_SO=$R/distributed_pytorch_example_amd/_C_dmabuiltin.so,DPE_AX_FWD=0,DPE_AX_BWD=0" MODEL=resnet50 ROUNDS=2 bash scripts/ab_bench.sh
