set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hgemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/hg_test.log 2>&1; rc=$?; tail -2 gpurun_out/hg_test.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_hgemm.py --square > gpurun_out/hg_sq.jsonl 2>&1 || exit 1
timeout -k 10 400 python -u scripts/bench_hgemm.py > gpurun_out/hg_bench.jsonl 2>&1 || exit 1
