#!/bin/bash
# Same-box per-kernel A/B: steady kernel traces of bench.py for the default build (A) and an alternative
# extension (B: DPE_EXT_SO=<path>), alternating.  bash scripts/gpu_ab_steady.sh <path-to-alt.so> [rounds]
# (path "-": the default build in both arms; BENV="VAR=val ..." adds an environment to the B arm)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/abs
ALT=$1; N=${2:-1}
cd /tmp && export TMPDIR=/tmp
for r in $(seq 1 $N); do
  for arm in A B; do
    rm -rf $R/gpurun_out/abs/tr
    if [ $arm = A ]; then
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/abs/tr -o run -- python3 $R/bench.py --steps 8 --warmup 3 ${BENCH_ARGS} > $R/gpurun_out/abs/$arm.log 2>&1 || { echo "$arm FAILED"; tail -20 $R/gpurun_out/abs/$arm.log; exit 1; }
    else
      if [ "$ALT" = "-" ]; then XS=""; else XS="DPE_EXT_SO=$ALT"; fi
      env $XS ${BENV} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/abs/tr -o run -- python3 $R/bench.py --steps 8 --warmup 3 ${BENCH_ARGS} > $R/gpurun_out/abs/$arm.log 2>&1 || { echo "$arm FAILED"; tail -20 $R/gpurun_out/abs/$arm.log; exit 1; }
    fi
    f=$(find $R/gpurun_out/abs/tr -name "*kernel_trace.csv" | head -1)
    python3 $R/scripts/prof_steady.py $f 4 ${MARK:-sgd_kernel} ${TOP:-80} > $R/gpurun_out/abs/steady_${arm}$r.txt
    echo "$arm$r $(head -1 $R/gpurun_out/abs/steady_${arm}$r.txt)"
    rm -rf $R/gpurun_out/abs/tr
  done
done
