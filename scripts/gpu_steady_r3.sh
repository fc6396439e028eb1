#!/bin/bash
# Fresh steady-state kernel breakdowns (ResNet-50 bs512, GPT-2) and the per-kernel hog factors.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/st
bash scripts/gpu_prof_steady.sh > gpurun_out/st/resnet.txt 2>&1 || { tail -20 gpurun_out/st/resnet.txt; exit 1; }
MARK=adam_kernel BENCH_ARGS="--model gpt2" bash scripts/gpu_prof_steady.sh > gpurun_out/st/gpt2.txt 2>&1 || { tail -20 gpurun_out/st/gpt2.txt; exit 1; }
head -50 gpurun_out/st/resnet.txt; head -40 gpurun_out/st/gpt2.txt
bash scripts/gpu_hog.sh 16 256 19968 136 > gpurun_out/st/hog.txt 2>&1 || { tail -20 gpurun_out/st/hog.txt; exit 1; }
grep -v "^{" gpurun_out/st/hog.txt | head -50
timeout -k 10 300 python -u scripts/sweep_wgrad_splits.py > gpurun_out/st/wgrad_splits.jsonl 2>&1 || { tail -20 gpurun_out/st/wgrad_splits.jsonl; exit 1; }; cat gpurun_out/st/wgrad_splits.jsonl
