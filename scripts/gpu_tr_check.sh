#!/bin/bash
# hgemm with compiler-invisible LDS-DMA: numerics, per-shape times, GPT-2 / ResNet-50 steps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/tr
timeout -k 10 300 python -u -m pytest tests/test_hgemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tr/pytest.log 2>&1 || { tail -30 gpurun_out/tr/pytest.log; exit 1; }
tail -1 gpurun_out/tr/pytest.log
timeout -k 10 300 python -u scripts/ab_hgemm_dynamic.py > gpurun_out/tr/ab_shapes.jsonl 2>&1 || { tail -20 gpurun_out/tr/ab_shapes.jsonl; exit 1; }
cat gpurun_out/tr/ab_shapes.jsonl
for m in gpt2 resnet50; do for i in 1 2; do timeout -k 10 240 python bench.py --model $m --steps 15 --warmup 4 > gpurun_out/tr/$m$i.log 2>&1 || { tail -20 gpurun_out/tr/$m$i.log; exit 1; }; tail -1 gpurun_out/tr/$m$i.log | cut -c1-160; done; done
