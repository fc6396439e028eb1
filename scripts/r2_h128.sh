# traffic probe: LDS-DMA conv A rows fetched as 128-B requests (numerically wrong variant) vs 64-B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=distributed_pytorch_example_amd
timeout -k 10 240 python -u scripts/bench_convs.py --batch 512 --miopen 0 --reps 10 > gpurun_out/h128_base.log 2>&1 || exit 1
DPE_EXT_SO=$PWD/$P/_C_h128.so timeout -k 10 240 python -u scripts/bench_convs.py --batch 512 --miopen 0 --reps 10 > gpurun_out/h128_var.log 2>&1 || exit 1
paste <(grep -v wgrad gpurun_out/h128_base.log | cut -c1-55) <(grep -v wgrad gpurun_out/h128_var.log | cut -c38-55)
