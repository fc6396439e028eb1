set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pw_test.log 2>&1; rc=$?; tail -1 gpurun_out/pw_test.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/pw_test.log | head; exit $rc; }
timeout -k 10 400 python scripts/bench_convs.py --batch 512 --reps 10 --miopen 0 > gpurun_out/convs_pw.txt 2>&1 || exit 1
DPE_PW_STREAM=0 timeout -k 10 400 python scripts/bench_convs.py --batch 512 --reps 10 --miopen 0 > gpurun_out/convs_nopw.txt 2>&1 || exit 1
paste <(grep fwd gpurun_out/convs_pw.txt | awk '{printf "%-24s %8s\n", $1$2$3$4$5, $7}') <(grep fwd gpurun_out/convs_nopw.txt | awk '{print $7}')
for i in 1 2; do
for v in 1 0; do
  DPE_PW_STREAM=$v timeout -k 10 200 python bench.py > gpurun_out/pw_step.log 2>&1 || exit 1
  echo "pw=$v step_ms=$(tail -1 gpurun_out/pw_step.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
done
