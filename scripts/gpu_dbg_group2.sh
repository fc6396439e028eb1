#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for reg in 0 1; do
  echo "== DPE_REGISTER_BUCKETS=$reg"
  DPE_REGISTER_BUCKETS=$reg DPE_WG_DEBUG=1 DPE_DEBUG_LOCAL=1 timeout -k 10 200 python -u -m pytest -x -q -s --timeout 150 --timeout-method thread -p no:cacheprovider \
    tests/test_ddp_rccl_world2_gpu.py::test_native_reducer_world2_rccl_gpt2 > gpurun_out/dbg2_$reg.log 2>&1
  grep -E "passed|failed" gpurun_out/dbg2_$reg.log | tail -1
  grep -E "vs avg|vs local|\[wg\] flushed" gpurun_out/dbg2_$reg.log | head -12 | cut -c1-220
done
grep -E "\[wg\]|\[ddp\]" gpurun_out/dbg2_1.log | head -60
exit 0
