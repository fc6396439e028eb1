#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/lay
timeout -k 10 300 python -u scripts/bench_hgemm_layouts.py > gpurun_out/lay/rates.jsonl 2>&1 || { tail -20 gpurun_out/lay/rates.jsonl; exit 1; }
cat gpurun_out/lay/rates.jsonl
bash scripts/gpu_pmc_hgemm.sh || exit 1
MARK=adam_kernel BENCH_ARGS="--model gpt2" bash scripts/gpu_prof_steady.sh > gpurun_out/lay/gpt2_steady.txt 2>&1 || { tail -20 gpurun_out/lay/gpt2_steady.txt; exit 1; }
head -32 gpurun_out/lay/gpt2_steady.txt
