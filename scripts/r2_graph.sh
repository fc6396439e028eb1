# HIP-graph replay of the whole step (bench.py --graph 1) vs eager, GPT-2 and ResNet-50; GPU suite first
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g_tests.log 2>&1 || { tail -30 gpurun_out/g_tests.log; exit 1; }
tail -1 gpurun_out/g_tests.log
for r in 1 2; do for v in 0 1; do
  timeout -k 10 300 python -u bench.py --model gpt2 --steps 30 --warmup 5 --graph $v > gpurun_out/gg.log 2>&1 || { tail -30 gpurun_out/gg.log; exit 1; }
  echo "gpt2 graph=$v $(tail -1 gpurun_out/gg.log | cut -c60-175)"
done; done
for r in 1 2; do for v in 0 1; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --graph $v > gpurun_out/gr.log 2>&1 || { tail -30 gpurun_out/gr.log; exit 1; }
  echo "r50 graph=$v $(tail -1 gpurun_out/gr.log | cut -c100-190)"
done; done
