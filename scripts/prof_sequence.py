#!/usr/bin/env python3
"""One steady step of a rocprofv3 kernel trace, kernel by kernel in launch order.

Prints index, duration (us), grid/workgroup sizes and the kernel name of every launch between
the K-th and (K+1)-th call of a per-step marker kernel -- for attributing an aggregated kernel
(e.g. bn_apply x 34) to the layers that launch it.
usage: prof_sequence.py trace.csv [skip_steps] [marker]
"""
import csv
import re
import sys

path = sys.argv[1]
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 3
marker = sys.argv[3] if len(sys.argv) > 3 else "sgd_kernel"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
marks = [r for r in rows if marker in r["Kernel_Name"]]
t0, t1 = int(marks[skip - 1]["End_Timestamp"]), int(marks[skip]["End_Timestamp"])
sel = [r for r in rows if t0 < int(r["Start_Timestamp"]) <= t1]
tot, prev_end, gaps = 0.0, t0, []
for i, r in enumerate(sel):
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    us = (en - st) / 1e3
    gap = max(0, st - prev_end) / 1e3  # idle time before this launch (ns -> us)
    prev_end = max(prev_end, en)
    tot += us
    grid = r.get("Grid_Size", r.get("Grid_Size_X", "?"))
    wg = r.get("Workgroup_Size", r.get("Workgroup_Size_X", "?"))
    name = re.sub(r"\(.*", "", r["Kernel_Name"])[:90]
    gaps.append((gap, i, name))
    print(f"{i:4d} {us:8.1f}us gap={gap:6.1f}us cum={tot / 1e3:7.3f}ms grid={grid:>8} wg={wg:>5} {name}")
print(f"# idle between launches: {sum(g for g, _, _ in gaps) / 1e3:.3f} ms over {len(gaps)} launches; largest:")
for g, i, n in sorted(gaps, reverse=True)[:12]:
    print(f"#   {g:7.1f}us before #{i} {n}")
