set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
for c in 0:256:0 32:256:32768; do
  tag=$(echo $c | tr ':' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/hogp_$tag -o run -- python3 scripts/hog_probe.py $c > gpurun_out/hogp_$tag.log 2>&1 || { tail -20 gpurun_out/hogp_$tag.log; exit 1; }
  f=$(find gpurun_out/hogp_$tag -name "*kernel_stats.csv" | head -1)
  python3 scripts/prof_summary.py $f 22 40 > gpurun_out/hogp_$tag.txt
  grep hog_blocks gpurun_out/hogp_$tag.log
done
