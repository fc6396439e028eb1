set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_ddp_rccl_world2_gpu.py tests/test_comm_gpu.py -x -v -s --timeout 150 --timeout-method thread > gpurun_out/w2_test.log 2>&1; rc=$?; grep -E "PASSED|FAILED|ok: world|registered|Error" gpurun_out/w2_test.log | head -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --force-comm --bucket-timing --steps 10 --warmup 3 > gpurun_out/r2_overlap_policy.log 2>&1 && tail -1 gpurun_out/r2_overlap_policy.log | cut -c1-600
