set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hgemm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/hg_test.log 2>&1; rc=$?; tail -25 gpurun_out/hg_test.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u scripts/bench_hgemm.py --check > gpurun_out/hg_bench.jsonl 2>&1; rc=$?; tail -3 gpurun_out/hg_bench.jsonl; exit $rc
