#!/bin/bash
# Round-6 end: full GPU suite, smoke, published single-GPU numbers, steady kernel breakdowns of both models.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || { tail -30 gpurun_out/final_tests.log; exit 1; }
tail -2 gpurun_out/final_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
bash scripts/gpu_published_numbers.sh || exit 1
bash scripts/gpu_prof_steady.sh > /dev/null || exit 1
cp gpurun_out/steady.txt gpurun_out/resnet50_steady_final.txt && head -3 gpurun_out/steady.txt
MARK=adam_kernel BENCH_ARGS="--model gpt2" bash scripts/gpu_prof_steady.sh > /dev/null || exit 1
cp gpurun_out/steady.txt gpurun_out/gpt2_steady_final.txt && head -3 gpurun_out/steady.txt
