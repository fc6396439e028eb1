# CU co-residency study on one GPU: RCCL kernel footprint at world 2, then the
# step time of ResNet-50 (and GPT-2) with RCCL-sized foreign workgroups resident during backward,
# with and without the compute side's CU budget, then per-kernel traces of the three modes.
# usage: bash scripts/gpu_hog.sh <hogs> <threads> <lds> <vgprs> <mode: 0 VALU-bound, 1 idle, 2 RCCL-like streaming>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/hog
NB=${1:-16}; TH=${2:-256}; LDS=${3:-20480}; VG=${4:-64}; MODE=${5:-0}
# WINDOWED=<GB/s>: hogs only in the modelled W = 8 bucket all-reduce windows (scripts/hog_probe.py --windowed)
H="--threads $TH --lds $LDS --vgprs $VG --sleepy $MODE --windowed ${WINDOWED:-0}"
cd $R
if [ "${TRACE_ONLY:-0}" != "1" ]; then
timeout -k 10 300 python3 scripts/hog_probe.py --model resnet50 $H --modes 0:0 $NB:0 $NB:$NB 0:$NB > gpurun_out/hog/rn.jsonl 2>&1 || { tail -20 gpurun_out/hog/rn.jsonl; exit 1; }
cat gpurun_out/hog/rn.jsonl
timeout -k 10 300 python3 scripts/hog_probe.py --model gpt2 $H --modes 0:0 $NB:0 $NB:$NB 0:$NB > gpurun_out/hog/gpt2.jsonl 2>&1 || { tail -20 gpurun_out/hog/gpt2.jsonl; exit 1; }
cat gpurun_out/hog/gpt2.jsonl
fi
cd /tmp && export TMPDIR=/tmp
for model in resnet50 gpt2; do
  mark=sgd_kernel; [ $model = gpt2 ] && mark=adam_kernel
  for m in 0:0 $NB:0 $NB:$NB; do
    tag=${model}_${m/:/_}
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/hog/t$tag -o run -- python3 $R/scripts/hog_probe.py --model $model $H --modes $m --rounds 1 --steps 5 > $R/gpurun_out/hog/t$tag.log 2>&1 || { tail -20 $R/gpurun_out/hog/t$tag.log; exit 1; }
  done
  f0=$(find $R/gpurun_out/hog/t${model}_0_0 -name "*kernel_trace.csv" | head -1)
  f1=$(find $R/gpurun_out/hog/t${model}_${NB}_0 -name "*kernel_trace.csv" | head -1)
  f2=$(find $R/gpurun_out/hog/t${model}_${NB}_${NB} -name "*kernel_trace.csv" | head -1)
  echo "== $model: no hogs -> $NB hogs, no CU budget"
  python3 $R/scripts/prof_compare.py $f0 $f1 $mark 5 20
  echo "== $model: no hogs -> $NB hogs, CU budget $NB"
  python3 $R/scripts/prof_compare.py $f0 $f2 $mark 5 20
  rm -f $f0 $f1 $f2
done
