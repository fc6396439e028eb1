#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv: per-step ms by kernel (grouped), top-N."""
import csv, re, sys
path = sys.argv[1]; steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot/1e6:.2f} ms ({tot/1e6/steps:.2f} ms/step over {steps:g} steps)")
def short(n):
    n = re.sub(r"\(.*", "", n)
    return n[:90]
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    t = float(r["TotalDurationNs"]) / 1e6
    print(f"{t/steps:7.3f} ms/step {100*float(r['TotalDurationNs'])/tot:5.1f}%  calls/step={int(r['Calls'])/steps:6.1f} avg={float(r['AverageNs'])/1e3:8.1f}us  {short(r['Name'])}")
