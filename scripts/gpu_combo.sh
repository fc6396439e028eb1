#!/bin/bash
# Several GPU steps in one call; a step that fails normally (exit 1) does not stop the call, a
# timeout / abort / segfault / kill does (no further GPU work after those).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/combo
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/gpurun_out/combo/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  case $rc in 124|137|134|139|-6|-11) echo "STOP after $name (rc $rc)"; tail -20 $R/gpurun_out/combo/$name.log; exit $rc;; esac
  return $rc
}
for step in "$@"; do
  case $step in
    prof) # steady ResNet-50 kernel trace (env passed through, e.g. DPE_BN3_GRAM)
          ( cd /tmp && export TMPDIR=/tmp && run prof_${PROF_TAG:-x} 300 rocprofv3 --kernel-trace --output-format csv \
              -d $R/gpurun_out/combo/prof_${PROF_TAG:-x} -o run -- python3 $R/bench.py --model ${PROF_MODEL:-resnet50} --steps 6 --warmup 3 ) || true
          f=$(find $R/gpurun_out/combo/prof_${PROF_TAG:-x} -name "*kernel_trace.csv" | head -1)
          python3 $R/scripts/prof_steady.py $f 3 ${PROF_MARK:-sgd_kernel} 60 > $R/gpurun_out/combo/steady_${PROF_TAG:-x}.txt && head -40 $R/gpurun_out/combo/steady_${PROF_TAG:-x}.txt
          python3 $R/scripts/prof_sequence.py $f 4 ${PROF_MARK:-sgd_kernel} > $R/gpurun_out/combo/sequence_${PROF_TAG:-x}.txt
          rm -f $f ;;
    convs) run convs 300 python -u scripts/bench_convs.py --batch 512 --miopen 0 --reps 10 --json gpurun_out/combo/convs_${PROF_TAG:-x}.jsonl
           tail -30 gpurun_out/combo/convs.log ;;
    parity0) run parity0 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
               tests/test_model_parity_gpu.py -k step0
             grep -E "PASSED|FAILED|% of bound|step-0|Error" $R/gpurun_out/combo/parity0.log | head -20 | cut -c1-200 ;;
    gpt2w2) run gpt2w2 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
              tests/test_ddp_rccl_world2_gpu.py tests/test_comm_gpu.py -k "gpt2 or world4"
            tail -3 gpurun_out/combo/gpt2w2.log ;;
    gram) run gram_tests 400 python -u -m pytest -v -s --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_bn3_gram_gpu.py
          grep -E "PASSED|FAILED|worst|Error" gpurun_out/combo/gram_tests.log | head -30 | cut -c1-220 ;;
    grambench) for arm in 0 1 0 1; do
            DPE_BN3_GRAM=$arm run bench_gram$arm 200 python bench.py --steps 20 --warmup 5 && \
              echo "gram=$arm $(tail -1 gpurun_out/combo/bench_gram$arm.log | cut -c1-110)"
          done ;;
    hconvab) for arm in 0 1 0 1; do
            DPE_HGEMM_CONV=$arm run bench_hconv$arm 200 python bench.py --steps 20 --warmup 5 && \
              echo "hconv=$arm $(tail -1 gpurun_out/combo/bench_hconv$arm.log | cut -c100-220)"
          done ;;
    hwgab) for arm in 0 1 0 1; do
            DPE_HGEMM_CONV_WGRAD=$arm run bench_hwg$arm 200 python bench.py --steps 20 --warmup 5 && \
              echo "hconv_wgrad=$arm $(tail -1 gpurun_out/combo/bench_hwg$arm.log | cut -c100-220)"
          done ;;
    bench) for i in 1 2; do
            run bench_r$i 200 python bench.py --steps 20 --warmup 5 && echo "run $i $(tail -1 gpurun_out/combo/bench_r$i.log | cut -c1-110)"
          done ;;
    gpt2bench) for arm in 0 2; do
            DPE_GPT2_WGRAD_GROUP=$arm run bench_gpt2_$arm 200 python bench.py --model gpt2 --steps 20 --warmup 5 && \
              echo "group=$arm $(tail -1 gpurun_out/combo/bench_gpt2_$arm.log | cut -c1-110)"
          done ;;
  esac
done
exit 0
