#!/bin/bash
# Dynamic GEMM schedule check on one GPU: hgemm numerics, A/B of the step time (dynamic vs static
# round-robin), and the RCCL-sized hog probe with and without it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/dyn
timeout -k 10 300 python -u -m pytest tests/test_hgemm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/dyn/pytest.log 2>&1 || { tail -30 gpurun_out/dyn/pytest.log; exit 1; }
tail -3 gpurun_out/dyn/pytest.log
ARMS="- DPE_HGEMM_DYNAMIC=0" MODEL=gpt2 ROUNDS=2 bash scripts/ab_bench.sh || exit 1
ARMS="- DPE_HGEMM_DYNAMIC=0" MODEL=resnet50 ROUNDS=2 bash scripts/ab_bench.sh || exit 1
H="--threads 256 --lds 19968 --vgprs 136"
for d in 1 0; do
  DPE_HGEMM_DYNAMIC=$d timeout -k 10 300 python3 scripts/hog_probe.py --model gpt2 $H --modes 0:0 16:0 16:16 > gpurun_out/dyn/hog_gpt2_d$d.jsonl 2>&1 || { tail -20 gpurun_out/dyn/hog_gpt2_d$d.jsonl; exit 1; }
  echo "dynamic=$d"; cat gpurun_out/dyn/hog_gpt2_d$d.jsonl
done
