#!/bin/bash
# Session start on a fresh box: the driver's GPU suite, smoke, both benches, and one ResNet-50
# steady step traced kernel by kernel (per-call attribution of the BN passes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/ss
[ "${SKIP_TESTS:-0}" = "1" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/ss/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/ss/pytest.log; exit 1; }
tail -2 gpurun_out/ss/pytest.log 2>/dev/null
[ "${SKIP_TESTS:-0}" = "1" ] || timeout -k 10 300 python -u -m pytest tests/test_model_parity_gpu.py -q -s --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/ss/parity.log 2>&1 || { tail -30 gpurun_out/ss/parity.log; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ss/smoke.log 2>&1 || { tail -20 gpurun_out/ss/smoke.log; exit 1; }
tail -1 gpurun_out/ss/smoke.log
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/ss/bench_resnet.log 2>&1 || { tail -20 gpurun_out/ss/bench_resnet.log; exit 1; }
tail -1 gpurun_out/ss/bench_resnet.log | cut -c1-200
timeout -k 10 240 python bench.py --model gpt2 --steps 20 --warmup 5 > gpurun_out/ss/bench_gpt2.log 2>&1 || { tail -20 gpurun_out/ss/bench_gpt2.log; exit 1; }
tail -1 gpurun_out/ss/bench_gpt2.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/ss/trace -o run -- python3 $R/bench.py --steps 6 --warmup 3 > $R/gpurun_out/ss/trace.log 2>&1 || { tail -20 $R/gpurun_out/ss/trace.log; exit 1; }
f=$(find $R/gpurun_out/ss/trace -name "*kernel_trace.csv" | head -1)
python3 $R/scripts/prof_steady.py $f 3 sgd_kernel 45 > $R/gpurun_out/ss/steady.txt
python3 $R/scripts/prof_sequence.py $f 4 sgd_kernel > $R/gpurun_out/ss/sequence.txt
head -3 $R/gpurun_out/ss/steady.txt
rm -f $f
