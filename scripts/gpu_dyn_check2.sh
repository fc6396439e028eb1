#!/bin/bash
# Per-shape and per-kernel A/B of the dynamic GEMM schedule (GPT-2 GEMMs; GPT-2 step traces).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/dyn
timeout -k 10 300 python -u -m pytest tests/test_hgemm_gpu.py -x -q --timeout 120 --timeout-method thread -k dynamic > gpurun_out/dyn/pytest2.log 2>&1 || { tail -30 gpurun_out/dyn/pytest2.log; exit 1; }
tail -1 gpurun_out/dyn/pytest2.log
timeout -k 10 300 python -u scripts/ab_hgemm_dynamic.py > gpurun_out/dyn/ab_shapes.jsonl 2>&1 || { tail -20 gpurun_out/dyn/ab_shapes.jsonl; exit 1; }
cat gpurun_out/dyn/ab_shapes.jsonl
ARMS="- DPE_HGEMM_DYNAMIC=0" MODEL=gpt2 ROUNDS=2 bash scripts/ab_bench.sh || exit 1
cd /tmp && export TMPDIR=/tmp
for d in 1 0; do
  DPE_HGEMM_DYNAMIC=$d timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/dyn/t$d -o run -- python3 $R/scripts/hog_probe.py --model gpt2 --modes 0:0 --rounds 1 --steps 5 > $R/gpurun_out/dyn/t$d.log 2>&1 || { tail -20 $R/gpurun_out/dyn/t$d.log; exit 1; }
done
f1=$(find $R/gpurun_out/dyn/t1 -name "*kernel_trace.csv" | head -1)
f0=$(find $R/gpurun_out/dyn/t0 -name "*kernel_trace.csv" | head -1)
echo "== static (A) -> dynamic (B)"
python3 $R/scripts/prof_compare.py $f0 $f1 adam_kernel 3 25
rm -f $f0 $f1
