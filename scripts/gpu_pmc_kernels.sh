#!/bin/bash
# Stall breakdown (one --pmc pass, kernel trace only) of the kernels a script launches:
#   [FILTER=substring] bash scripts/gpu_pmc_kernels.sh <script.py> [args...]   -> gpurun_out/pmck/summary.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/pmck
cd /tmp && export TMPDIR=/tmp
S=$1; shift
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS \
  --kernel-trace --output-format csv -d $R/gpurun_out/pmck/a -o run -- python3 $R/$S "$@" \
  > $R/gpurun_out/pmck/a.log 2>&1 || { echo "pass a failed"; tail -5 $R/gpurun_out/pmck/a.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM \
  --kernel-trace --output-format csv -d $R/gpurun_out/pmck/b -o run -- python3 $R/$S "$@" \
  > $R/gpurun_out/pmck/b.log 2>&1 || { echo "pass b failed"; tail -5 $R/gpurun_out/pmck/b.log; exit 1; }
python3 - $R/gpurun_out/pmck <<'PY' | tee $R/gpurun_out/pmck/summary.txt
import collections, csv, glob, sys
root = sys.argv[1]
per = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "?").split("(")[0]
        per[k][row["Counter_Name"]] += float(row["Counter_Value"])
import os
flt = os.environ.get("FILTER", "")
rows = sorted([kv for kv in per.items() if flt in kv[0]], key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:int(os.environ.get("TOPK", "14"))]
for k, c in rows:
    wc = c.get("SQ_WAVE_CYCLES", 1) or 1
    print(k[:100])
    print("   " + "  ".join(f"{n}={v:.4g}" for n, v in sorted(c.items())))
    print(f"   wait%={100*c.get('SQ_WAIT_ANY',0)/wc:.1f} waitinst%={100*c.get('SQ_WAIT_INST_ANY',0)/wc:.1f} active%={100*c.get('SQ_ACTIVE_INST_ANY',0)/wc:.1f}")
PY
find $R/gpurun_out/pmck -name "*.csv" -size +20M -delete
