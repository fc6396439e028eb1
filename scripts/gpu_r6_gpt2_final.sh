#!/bin/bash
# GPT-2 steady kernel breakdown and two bench runs at HEAD (after the LayerNorm changes).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2; do
  timeout -k 10 200 python bench.py --model gpt2 --steps 20 --warmup 5 > gpurun_out/g2.log 2>&1 || { tail -5 gpurun_out/g2.log; exit 1; }
  echo "gpt2_$i $(grep '"metric"' gpurun_out/g2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/step", round(d["value"]), d["unit"])')"
done
MARK=adam_kernel BENCH_ARGS="--model gpt2" bash scripts/gpu_prof_steady.sh > /dev/null || exit 1
cp gpurun_out/steady.txt gpurun_out/gpt2_steady_final.txt && head -3 gpurun_out/steady.txt
