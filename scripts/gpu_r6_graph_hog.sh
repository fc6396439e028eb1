set -o pipefail
mkdir -p gpurun_out/ab
for r in 1 2 3; do for g in 0 1; do
 timeout -k 10 240 python bench.py --steps 20 --warmup 5 --graph $g > gpurun_out/ab/graph$g.log 2>&1 || { echo FAIL; tail -5 gpurun_out/ab/graph$g.log; exit 1; }
 echo "r$r graph=$g $(tail -1 gpurun_out/ab/graph$g.log | cut -c150-230)"
done; done
bash scripts/gpu_hog_table.sh > gpurun_out/hogtab.txt 2>&1; tail -30 gpurun_out/hogtab.txt
