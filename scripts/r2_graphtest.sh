set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -v --timeout 150 --timeout-method thread -k "graph or counts" > gpurun_out/gt.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/gt.log | head -30; tail -40 gpurun_out/gt.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/gt.log
