#!/bin/bash
# LDS counters of the persistent GEMM per operand layout (one pass of <= 8 SQ counters).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/pmc/a -o run -- python3 $R/scripts/pmc_hgemm_layouts.py > $R/gpurun_out/pmc/a.log 2>&1 || { tail -20 $R/gpurun_out/pmc/a.log; exit 1; }
f=$(find $R/gpurun_out/pmc/a -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections, re
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"]
    if "hgemm_kernel" not in k:
        continue
    m = re.search(r"hgemm_kernel<([^>]*)>", k)
    key = m.group(1) if m else k[:60]
    agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(key, r["Counter_Name"])] += 1
for key, d in agg.items():
    n = max(cnt[(key, c)] for c in d)
    print(key, {c: round(v / n) for c, v in sorted(d.items())})
PY
