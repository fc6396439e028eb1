set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/bnu_test.log 2>&1; rc=$?; tail -1 gpurun_out/bnu_test.log; [ $rc -ne 0 ] && exit $rc
for nb in 1024 2048 4096 1024 2048; do
  export DPE_BN_NB=$nb
  timeout -k 10 200 python bench.py > gpurun_out/bnu_step.log 2>&1 || exit 1
  echo "nb=$nb step_ms=$(tail -1 gpurun_out/bnu_step.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
