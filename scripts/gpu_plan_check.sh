#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/plan
timeout -k 10 300 python -u scripts/sweep_wgrad_splits.py > gpurun_out/plan/splits.jsonl 2>&1 || { tail -20 gpurun_out/plan/splits.jsonl; exit 1; }
cat gpurun_out/plan/splits.jsonl
ARMS="- DPE_HGEMM_PLAN2=0" MODEL=gpt2 ROUNDS=2 bash scripts/ab_bench.sh || exit 1
