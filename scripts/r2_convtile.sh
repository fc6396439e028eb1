set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python scripts/bench_convs.py --batch 512 --reps 10 --miopen 0 > gpurun_out/convs_auto.txt 2>&1 || exit 1
DPE_DMA_TILE=256x128 timeout -k 10 400 python scripts/bench_convs.py --batch 512 --reps 10 --miopen 0 > gpurun_out/convs_256x128.txt 2>&1 || exit 1
paste gpurun_out/convs_auto.txt gpurun_out/convs_256x128.txt | grep "fwd" | awk '{print $1,$2,$3,$4,$5,$6, "|", $8, $11}'
tail -2 gpurun_out/convs_auto.txt; tail -2 gpurun_out/convs_256x128.txt
