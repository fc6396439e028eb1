#!/usr/bin/env python3
"""RCCL kernel footprint from a rocprofv3 kernel trace of one rank: per RCCL kernel name the grid
(workgroups = channel blocks), workgroup size, VGPRs / LDS, call count and duration quantiles, plus the
bench line's bucket layout.  usage: rccl_kernels.py kernel_trace.csv [bench.json]"""
import collections
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
agg = collections.OrderedDict()
for r in rows:
    n = r["Kernel_Name"]
    if "nccl" not in n.lower() and "rccl" not in n.lower():
        continue
    wg = int(r.get("Workgroup_Size", r.get("Workgroup_Size_X", 0)) or 0)
    grid = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
    key = (n.split("(")[0][:80], grid // max(wg, 1), wg, r.get("VGPR_Count", r.get("Arch_VGPR_Count", "?")),
           r.get("LDS_Block_Size", r.get("Group_Segment_Size", "?")))
    agg.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print("RCCL kernels on rank 0 (name | workgroups = channel blocks | threads/WG | VGPRs | LDS B | calls | "
      "duration us min / median / max)")
for (n, blocks, wg, vg, lds), ds in agg.items():
    ds.sort()
    print(f"  {n} | {blocks} | {wg} | {vg} | {lds} | {len(ds)} | {ds[0]:.1f} / {ds[len(ds) // 2]:.1f} / {ds[-1]:.1f}")
if len(sys.argv) > 2:
    line = json.loads(open(sys.argv[2]).read())
    print("bench:", {k: line[k] for k in ("value", "unit", "n_gpus", "ms_per_step", "config")})
    b = line.get("buckets") or {}
    print(f"buckets: {b.get('count')} (comm {b.get('comm_ms')} ms, overlap {b.get('overlap_pct')} %):",
          [(x["bucket"], round(x["bytes"] / 2**20, 2)) for x in b.get("per_bucket", [])])
