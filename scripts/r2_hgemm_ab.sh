set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hgemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/hg_test.log 2>&1; rc=$?; tail -3 gpurun_out/hg_test.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/bench_hgemm.py --square > gpurun_out/hg_sq_new.jsonl 2>&1 || exit 1
DPE_EXT_SO=$PWD/distributed_pytorch_example_amd/_C_sched0.so timeout -k 10 300 python -u scripts/bench_hgemm.py --square > gpurun_out/hg_sq_old.jsonl 2>&1 || exit 1
timeout -k 10 400 python -u scripts/bench_hgemm.py --check > gpurun_out/hg_bench.jsonl 2>&1 || exit 1
