#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
DPE_WG_DEBUG=1 DPE_DEBUG_LOCAL=1 timeout -k 10 200 python -u -m pytest -x -q -s --timeout 150 --timeout-method thread -p no:cacheprovider \
  tests/test_ddp_rccl_world2_gpu.py::test_native_reducer_world2_rccl_gpt2 > gpurun_out/dbg2.log 2>&1
grep -E "vs avg|vs local|\[wg\]|\[ddp\]" gpurun_out/dbg2.log | head -80
exit 0
