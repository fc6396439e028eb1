# GPU suite + smoke + ResNet-50 and GPT-2 benches (current tree)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/verify_tests.log 2>&1 || { tail -30 gpurun_out/verify_tests.log; exit 1; }
tail -2 gpurun_out/verify_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/verify_smoke.log 2>&1 || { tail -20 gpurun_out/verify_smoke.log; exit 1; }
tail -1 gpurun_out/verify_smoke.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/verify_bench.log 2>&1 || exit 1
  tail -1 gpurun_out/verify_bench.log | cut -c1-200
done
timeout -k 10 300 python -u bench.py --model gpt2 --steps 20 --warmup 5 > gpurun_out/verify_gpt2.log 2>&1 || exit 1
tail -1 gpurun_out/verify_gpt2.log | cut -c1-200
