set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r2_gputest.log 2>&1; rc=$?; tail -1 gpurun_out/r2_gputest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED|^E " gpurun_out/r2_gputest.log | head -30; exit $rc; fi
for i in 1 2; do
for v in 1 0; do
  DPE_PW_STREAM=$v timeout -k 10 200 python bench.py > gpurun_out/pw_step.log 2>&1 || exit 1
  echo "pw=$v step_ms=$(tail -1 gpurun_out/pw_step.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
done
