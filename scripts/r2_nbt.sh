# one num_batches_tracked launch per step: model tests, bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/nbt_tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/nbt_tests.log | head -30; tail -30 gpurun_out/nbt_tests.log; exit 1; }
tail -1 gpurun_out/nbt_tests.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/nbt.log 2>&1 || exit 1
  echo "r50 $(tail -1 gpurun_out/nbt.log | cut -c100-175)"
done
