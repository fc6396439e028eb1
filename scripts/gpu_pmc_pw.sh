#!/bin/bash
# Stall breakdown of the streaming pointwise kernels over bench steps (one --pmc pass, kernel trace only).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/pmcpw
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS \
  --kernel-trace --output-format csv -d $R/gpurun_out/pmcpw/a -o run -- python3 $R/bench.py --steps 2 --warmup 1 \
  > $R/gpurun_out/pmcpw/a.log 2>&1 || { echo "pass a failed"; tail -5 $R/gpurun_out/pmcpw/a.log; exit 1; }
python3 - $R/gpurun_out/pmcpw/a <<'PY'
import collections, csv, glob, sys
root = sys.argv[1]
per = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "?").split("(")[0]
        per[k][row["Counter_Name"]] += float(row["Counter_Value"])
rows = sorted(per.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:16]
print(f"{'wave-cyc':>10} {'wait%':>6} {'waitinst%':>9} {'active%':>8} {'valu/wave-kcyc':>14} {'vmem':>8} {'lds':>8}  kernel")
for k, c in rows:
    wc = c.get("SQ_WAVE_CYCLES", 1) or 1
    print(f"{wc:10.3g} {100*c.get('SQ_WAIT_ANY',0)/wc:6.1f} {100*c.get('SQ_WAIT_INST_ANY',0)/wc:9.1f} {100*c.get('SQ_ACTIVE_INST_ANY',0)/wc:8.1f} "
          f"{1000*c.get('SQ_INSTS_VALU',0)/wc:14.2f} {c.get('SQ_INSTS_VMEM',0):8.3g} {c.get('SQ_INSTS_LDS',0):8.3g}  {k[:90]}")
PY
find $R/gpurun_out/pmcpw -name "*.csv" -size +20M -delete
