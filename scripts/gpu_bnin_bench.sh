#!/bin/bash
# bench_bnin.py under the DPE_AX_DBG experiment switches (0 = the real kernel)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/bnin
for d in ${DBGS:-0 1 3 7}; do
  DPE_AX_DBG=$d timeout -k 10 200 python -u scripts/bench_bnin.py > gpurun_out/bnin/dbg$d.jsonl 2>&1 || { tail -20 gpurun_out/bnin/dbg$d.jsonl; exit 1; }
  echo "== DPE_AX_DBG=$d"; cat gpurun_out/bnin/dbg$d.jsonl
done
