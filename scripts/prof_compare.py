#!/usr/bin/env python3
"""Per-kernel time of two rocprofv3 kernel traces of the same workload (e.g. scripts/hog_probe.py
with and without foreign workgroups): ms per step of each kernel in A and B and their ratio.
Steps are delimited by a marker kernel (one launch per step); the first `skip` steps are dropped.

usage: prof_compare.py a_kernel_trace.csv b_kernel_trace.csv [marker] [skip] [topN]"""
import collections
import csv
import re
import sys


def load(path, marker, skip):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [r for r in rows if marker in r["Kernel_Name"]]
    t0, t1 = int(marks[skip - 1]["End_Timestamp"]), int(marks[-1]["End_Timestamp"])
    steps = len(marks) - skip
    agg = collections.defaultdict(float)
    for r in rows:
        if t0 < int(r["Start_Timestamp"]) <= t1 and "hog" not in r["Kernel_Name"]:
            agg[re.sub(r"\(.*", "", r["Kernel_Name"])[:90]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    return {k: v / steps for k, v in agg.items()}, (t1 - t0) / 1e6 / steps


a, wa = load(sys.argv[1], sys.argv[3] if len(sys.argv) > 3 else "sgd_kernel", int(sys.argv[4]) if len(sys.argv) > 4 else 2)
b, wb = load(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "sgd_kernel", int(sys.argv[4]) if len(sys.argv) > 4 else 2)
top = int(sys.argv[5]) if len(sys.argv) > 5 else 25
print(f"wall ms/step  A {wa:.3f}  B {wb:.3f}  ({wb / wa:.3f}x)")
print(f"kernel-busy   A {sum(a.values()):.3f}  B {sum(b.values()):.3f}")
keys = sorted(set(a) | set(b), key=lambda k: -abs(b.get(k, 0) - a.get(k, 0)))
for k in keys[:top]:
    x, y = a.get(k, 0.0), b.get(k, 0.0)
    print(f"{y - x:+.3f}  {x:7.3f} -> {y:7.3f}  x{(y / x if x else float('inf')):.2f}  {k}")
