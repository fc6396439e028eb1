#!/usr/bin/env python3
"""Largest idle gaps between consecutive kernels in a rocprofv3 kernel trace (steady window: after the first
`mark` kernel), with the kernels on either side.  usage: trace_gaps.py trace.csv [mark] [top]"""
import csv
import sys

f = sys.argv[1]
mark = sys.argv[2] if len(sys.argv) > 2 else "adam_kernel"
top = int(sys.argv[3]) if len(sys.argv) > 3 else 15
rows = []
with open(f) as fh:
    for r in csv.DictReader(fh):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
start = next((i for i, r in enumerate(rows) if mark in r[2]), 0)
rows = rows[start:]
gaps = []
end = rows[0][1]
for i in range(1, len(rows)):
    g = rows[i][0] - end
    if g > 0:
        gaps.append((g, rows[i - 1][2][:70], rows[i][2][:70]))
    end = max(end, rows[i][1])
gaps.sort(reverse=True)
print(f"{len(rows)} kernels, total gap {sum(g for g, *_ in gaps) / 1e3:.1f} us")
for g, a, b in gaps[:top]:
    print(f"{g / 1e3:8.1f} us  after {a}  ->  {b}")
