#!/bin/bash
# Streaming pointwise-conv change: numerics, ResNet-50 step, steady profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/pw
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 150 --timeout-method thread -k "pw or stream or resnet or bitwise or pointwise" > gpurun_out/pw/pytest.log 2>&1 || { tail -30 gpurun_out/pw/pytest.log; exit 1; }
tail -1 gpurun_out/pw/pytest.log
for i in 1 2; do timeout -k 10 240 python bench.py --steps 15 --warmup 4 > gpurun_out/pw/bench$i.log 2>&1 || { tail -20 gpurun_out/pw/bench$i.log; exit 1; }; tail -1 gpurun_out/pw/bench$i.log | cut -c1-200; done
bash scripts/gpu_prof_steady.sh > gpurun_out/pw/steady.txt 2>&1 || { tail -20 gpurun_out/pw/steady.txt; exit 1; }
grep -E "pw_stream|steady steps" gpurun_out/pw/steady.txt
