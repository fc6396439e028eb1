#!/bin/bash
# Targeted GPU tests (TESTS=...) then the ResNet-50 / GPT-2 benches and a ResNet steady trace.
set -o pipefail
mkdir -p gpurun_out/chk
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider ${TESTS} > gpurun_out/chk/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "^E |Error|FAILED" gpurun_out/chk/tests.log | head -30; exit 1; }
tail -1 gpurun_out/chk/tests.log
for m in ${MODELS:-resnet50 gpt2}; do
  timeout -k 10 200 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/chk/bench_$m.log 2>&1 || { tail -20 gpurun_out/chk/bench_$m.log; exit 1; }
  grep '"metric"' gpurun_out/chk/bench_$m.log | python3 -c 'import json,sys; l=json.loads(sys.stdin.read()); print(l["config"]["model"], l["value"], l["ms_per_step"])'
done
if [ "${TRACE:-1}" = "1" ]; then bash scripts/gpu_prof_steady.sh > /dev/null && head -3 gpurun_out/steady.txt; fi
