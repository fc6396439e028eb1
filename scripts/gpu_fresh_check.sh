#!/bin/bash
# Overwrite-first-write gradient protocol: equivalence test, DDP/model GPU tests, GPT-2 A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/fresh
timeout -k 10 600 python -u -m pytest tests/test_comm_gpu.py tests/test_models_gpu.py tests/test_hgemm_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/fresh/pytest.log 2>&1 || { tail -30 gpurun_out/fresh/pytest.log; exit 1; }
tail -1 gpurun_out/fresh/pytest.log
ARMS="- DPE_GRAD_FRESH=0" MODEL=gpt2 ROUNDS=3 bash scripts/ab_bench.sh || exit 1
