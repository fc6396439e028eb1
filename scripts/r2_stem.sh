# A/B: s2d stem conv on the 256x64 2-stage tile (DPE_STEM_W64=1) vs 128x64
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do for v in 0 1; do
  DPE_STEM_W64=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/stem.log 2>&1 || exit 1
  echo "stem_w64=$v $(tail -1 gpurun_out/stem.log | cut -c100-190)"
done; done
for v in 0 1; do
  DPE_STEM_W64=$v timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_stem$v -o run -- python bench.py --steps 6 --warmup 3 > gpurun_out/prof_stem$v.log 2>&1 || exit 1
done
