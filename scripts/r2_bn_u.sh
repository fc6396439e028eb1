set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/bnu_test.log 2>&1; rc=$?; tail -1 gpurun_out/bnu_test.log; [ $rc -ne 0 ] && exit $rc
for cfg in "1 1 1" "1 2 2" "1 4 4" "2 2 2" "1 2 2" "1 1 1"; do
  set -- $cfg
  export DPE_BN_U_APPLY=$1 DPE_BN_U_APPLY2=$2 DPE_BN_U_BWD=$3
  timeout -k 10 200 python scripts/bench_bn.py > gpurun_out/bnu_$1$2$3.txt 2>&1 || exit 1
  timeout -k 10 200 python bench.py > gpurun_out/bnu_step.log 2>&1 || exit 1
  echo "U=$cfg step_ms=$(tail -1 gpurun_out/bnu_step.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])') bwd_apply_us=$(grep bwd_apply gpurun_out/bnu_$1$2$3.txt | awk '{printf "%s ", $4}')"
done
