#!/bin/bash
# Same-box A/B of the optimizer-in-backward path (bench.py --overlap-optimizer), alternating processes.
set -o pipefail
mkdir -p gpurun_out/ab
for model in ${MODELS:-gpt2 resnet50}; do
  for rep in 1 2; do
    for ov in 0 1; do
      timeout -k 10 200 python bench.py --model $model --steps 20 --warmup 5 --overlap-optimizer $ov > gpurun_out/ab/$model.$ov.$rep.log 2>&1 || { tail -20 gpurun_out/ab/$model.$ov.$rep.log; exit 1; }
      echo "$model overlap=$ov rep=$rep $(grep '"metric"' gpurun_out/ab/$model.$ov.$rep.log | python3 -c 'import json,sys; l=json.loads(sys.stdin.read()); print(l["value"], l["ms_per_step"])')"
    done
  done
done
