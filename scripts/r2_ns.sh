# A/B: DMA ring depth of the 4-wave conv tiles (compile-time variants loaded with DPE_EXT_SO)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=distributed_pytorch_example_amd
for v in _C.so _C_ns8k.so _C_ns16k.so; do
  DPE_EXT_SO=$PWD/$P/$v timeout -k 10 240 python -u scripts/bench_convs.py --batch 512 --miopen 0 --reps 10 > gpurun_out/ns_convs_$v.log 2>&1 || exit 1
  echo "$v $(tail -2 gpurun_out/ns_convs_$v.log | head -1)"
done
for r in 1 2; do for v in _C.so _C_ns8k.so _C_ns16k.so; do
  DPE_EXT_SO=$PWD/$P/$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/ns_bench.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/ns_bench.log | cut -c1-150)"
done; done
