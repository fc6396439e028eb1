# fused CE (VALU-trimmed row-in-registers kernel): numerics, kernel time, GPT-2 step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "cross_entropy or gpt2 or simplenet" > gpurun_out/ce_tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/ce_tests.log | head -30; tail -30 gpurun_out/ce_tests.log; exit 1; }
tail -1 gpurun_out/ce_tests.log
timeout -k 10 120 python -u scripts/ce_bench.py 2>&1 | grep -v amdgpu.ids
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --model gpt2 --steps 30 --warmup 5 > gpurun_out/ceg.log 2>&1 || exit 1
  echo "$(tail -1 gpurun_out/ceg.log | cut -c60-175)"
done
