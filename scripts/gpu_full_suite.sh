#!/bin/bash
# The whole GPU test suite (one process), as the driver runs it at round end.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/suite
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  --deselect tests/test_model_parity_gpu.py > gpurun_out/suite/pytest.log 2>&1
rc=$?
tail -15 gpurun_out/suite/pytest.log
exit $rc
