# a2 on load also for the 128-channel (layer-2) bottlenecks: full GPU suite, then A/B of the channel cap
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/a2b_tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/a2b_tests.log | head -30; tail -30 gpurun_out/a2b_tests.log; exit 1; }
tail -1 gpurun_out/a2b_tests.log
for r in 1 2 3; do for v in 64 128; do
  DPE_PW_BNIN_CMAX=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/a2b.log 2>&1 || exit 1
  echo "pw_bnin_cmax=$v $(tail -1 gpurun_out/a2b.log | cut -c100-175)"
done; done
