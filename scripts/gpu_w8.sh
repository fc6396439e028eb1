set -o pipefail
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r5a.log 2>&1 && tail -1 gpurun_out/bench_r5a.log | cut -c1-220 &&
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_ddp_rccl_world2_gpu.py -k world8 > gpurun_out/w8_tests.log 2>&1; tail -3 gpurun_out/w8_tests.log;
grep -E "ok: world-8|survivors" gpurun_out/w8_tests.log | head -3
