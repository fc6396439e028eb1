#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/dbg
for r in 16 0; do timeout -k 10 200 python -u scripts/debug_bn_repro.py $r > gpurun_out/dbg/r$r.log 2>&1 || { tail -20 gpurun_out/dbg/r$r.log; exit 1; }; echo "reserve $r"; grep -v amdgpu.ids gpurun_out/dbg/r$r.log; done
DPE_HGEMM_DYNAMIC=0 timeout -k 10 200 python -u scripts/debug_bn_repro.py 16 > gpurun_out/dbg/nodyn.log 2>&1 || { tail -20 gpurun_out/dbg/nodyn.log; exit 1; }; echo "reserve 16, static hgemm"; grep -v amdgpu.ids gpurun_out/dbg/nodyn.log
