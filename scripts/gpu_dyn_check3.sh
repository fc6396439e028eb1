#!/bin/bash
# Dynamic GEMM schedule: numerics, per-shape A/B (idle and with a CU budget), GPT-2 / ResNet A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/dyn
timeout -k 10 300 python -u -m pytest tests/test_hgemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dyn/pytest3.log 2>&1 || { tail -30 gpurun_out/dyn/pytest3.log; exit 1; }
tail -1 gpurun_out/dyn/pytest3.log
timeout -k 10 300 python -u scripts/ab_hgemm_dynamic.py > gpurun_out/dyn/ab_shapes3.jsonl 2>&1 || { tail -20 gpurun_out/dyn/ab_shapes3.jsonl; exit 1; }
cat gpurun_out/dyn/ab_shapes3.jsonl
ARMS="- DPE_HGEMM_DYNAMIC=0" MODEL=gpt2 ROUNDS=2 bash scripts/ab_bench.sh || exit 1
