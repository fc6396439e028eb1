set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_optim_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/optim_test.log 2>&1; rc=$?; grep -E "PASSED|FAILED|Error|assert" gpurun_out/optim_test.log | head -30; exit $rc
