#!/bin/bash
# Re-measure the published single-GPU configs: ResNet-50 batch 512 / 256,
# grad-accum 8, GPT-2-small.  One process per run, results to gpurun_out/pub/.
set -o pipefail
mkdir -p gpurun_out/pub
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/pub/$n.log 2>&1 || { echo "$n FAILED"; tail -20 gpurun_out/pub/$n.log; exit 1; }
  echo "$n $(grep "\"metric\"" gpurun_out/pub/$n.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/step", round(d["value"]), d["unit"])')"
}
run gpt2_a --model gpt2 --steps 20 --warmup 5
run resnet512 --steps 20 --warmup 5
run resnet256 --batch-size 256 --steps 20 --warmup 5
run accum8 --grad-accum 8 --steps 4 --warmup 1
run gpt2_b --model gpt2 --steps 20 --warmup 5
