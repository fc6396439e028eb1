# A/B: 256x64 4x1-wave tile with a 2-stage ring for the N = 64 convs (layer 1), forced via DPE_DMA_TILE
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=distributed_pytorch_example_amd
timeout -k 10 240 python -u scripts/bench_convs.py --batch 512 --miopen 0 --reps 10 > gpurun_out/w64_base.log 2>&1 || exit 1
DPE_EXT_SO=$PWD/$P/_C_w64.so DPE_DMA_TILE=256x128 timeout -k 10 240 python -u scripts/bench_convs.py --batch 512 --miopen 0 --reps 10 > gpurun_out/w64_var.log 2>&1 || exit 1
DPE_DMA_TILE=256x128 timeout -k 10 240 python -u scripts/bench_convs.py --batch 512 --miopen 0 --reps 10 > gpurun_out/w64_ns3.log 2>&1 || exit 1
for f in base var ns3; do echo "== $f"; grep -E "^\((8|64|256), (64|256), .*56|224" gpurun_out/w64_$f.log | grep -v wgrad; done
