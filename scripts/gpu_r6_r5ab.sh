#!/bin/bash
# Same-box A/B of the whole framework: the round-5 final commit (f422de3, worktree abso/r5tree with its own
# in-tree build) vs HEAD, ResNet-50 (bench default) and GPT-2, alternating processes.
set -o pipefail
R=$GRAFT_REPO_ROOT
one() {  # dir model
  (cd $1 && timeout -k 10 200 python bench.py --model $2 --steps 20 --warmup 5 > $R/gpurun_out/r5ab.log 2>&1) || { tail -5 $R/gpurun_out/r5ab.log; exit 1; }
  grep '"metric"' $R/gpurun_out/r5ab.log | python3 -c 'import json,sys; l=json.loads(sys.stdin.read()); print(l["value"], l["ms_per_step"])'
}
for m in resnet50 gpt2; do
  for r in 1 2 3; do
    echo "$m r5   $(one $R/abso/r5tree $m)"
    echo "$m head $(one $R $m)"
  done
done
