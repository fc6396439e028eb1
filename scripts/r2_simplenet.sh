set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_simplenet_parity_gpu.py tests/test_models_gpu.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/sn_test.log 2>&1; rc=$?; grep -E "PASSED|FAILED|Error|assert|loss curve" gpurun_out/sn_test.log | head -40; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python bench.py --model simplenet --steps 50 --warmup 10 > gpurun_out/sn_bench.log 2>&1 && tail -1 gpurun_out/sn_bench.log
timeout -k 10 120 python bench.py --model simplenet --steps 50 --warmup 10 --dtype bf16 > gpurun_out/sn_bench16.log 2>&1 && tail -1 gpurun_out/sn_bench16.log
