# GPU suite + ResNet-50 bench (current tree)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/verify_tests.log 2>&1 || { tail -30 gpurun_out/verify_tests.log; exit 1; }
tail -2 gpurun_out/verify_tests.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/verify_bench.log 2>&1 || exit 1
  tail -1 gpurun_out/verify_bench.log | cut -c1-200
done
