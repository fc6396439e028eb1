#!/bin/bash
# Counters over the benchmarked steady steps: two --pmc passes per model (TCC slots:
# FETCH_SIZE 3, WRITE_SIZE 2 -> separate passes), kernel-trace only beside --pmc (pool rules).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/pmcs
cd /tmp && export TMPDIR=/tmp
for model in resnet50 gpt2; do
  timeout -s KILL 240 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE FETCH_SIZE \
    --kernel-trace --output-format csv -d $R/gpurun_out/pmcs/${model}_a -o run -- python3 $R/bench.py --model $model --steps 3 --warmup 2 \
    > $R/gpurun_out/pmcs/${model}_a.log 2>&1 || { echo "pass a failed ($model)"; tail -5 $R/gpurun_out/pmcs/${model}_a.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d $R/gpurun_out/pmcs/${model}_b -o run -- python3 $R/bench.py --model $model --steps 3 --warmup 2 \
    > $R/gpurun_out/pmcs/${model}_b.log 2>&1 || { echo "pass b failed ($model)"; tail -5 $R/gpurun_out/pmcs/${model}_b.log; exit 1; }
  python3 $R/scripts/pmc_steady_summary.py $R/gpurun_out/pmcs/${model}_a $R/gpurun_out/pmcs/${model}_b $model ${TOPN:-12} \
    > $R/gpurun_out/pmcs/${model}_summary.txt && cat $R/gpurun_out/pmcs/${model}_summary.txt
  mark=sgd_kernel; [ $model = gpt2 ] && mark=adam_kernel
  python3 $R/scripts/pmc_dispatch_step.py $R/gpurun_out/pmcs/${model}_a $R/gpurun_out/pmcs/${model}_b $mark 0 \
    > $R/gpurun_out/pmcs/${model}_dispatch.txt || echo "(per-dispatch table failed)"
  find $R/gpurun_out/pmcs -name "*.csv" -size +20M -delete
done
