# full GPU suite + smoke + benches + steady-state profiles, then the wgrad block-target A/B (512 vs default 768)
set -o pipefail
bash scripts/r2_final.sh || exit 1
for r in 1 2 3; do for v in 512 768; do
  DPE_WGRAD_BLOCKS=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/wb.log 2>&1 || exit 1
  echo "wgrad_blocks=$v $(tail -1 gpurun_out/wb.log | cut -c100-190)"
done; done
