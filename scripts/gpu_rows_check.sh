#!/bin/bash
# Row-walking kernels with the CU-budget grid: numerics, ResNet A/B, hog per-kernel factors.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/rows
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread -k "row or stem" > gpurun_out/rows/pytest.log 2>&1 || { tail -30 gpurun_out/rows/pytest.log; exit 1; }
tail -2 gpurun_out/rows/pytest.log
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 150 --timeout-method thread -k "bitwise or resnet" > gpurun_out/rows/pytest_models.log 2>&1 || { tail -30 gpurun_out/rows/pytest_models.log; exit 1; }
tail -2 gpurun_out/rows/pytest_models.log
for i in 1 2; do timeout -k 10 240 python bench.py --steps 15 --warmup 4 > gpurun_out/rows/bench$i.log 2>&1 || { tail -20 gpurun_out/rows/bench$i.log; exit 1; }; tail -1 gpurun_out/rows/bench$i.log | cut -c1-200; done
bash scripts/gpu_hog.sh 16 256 19968 136 > gpurun_out/rows/hog.txt 2>&1 || { tail -20 gpurun_out/rows/hog.txt; exit 1; }
grep -v "^{" gpurun_out/rows/hog.txt | head -50
