set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_ddp_rccl_world2_gpu.py tests/test_comm_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/w2_test.log 2>&1; rc=$?; tail -30 gpurun_out/w2_test.log; exit $rc
