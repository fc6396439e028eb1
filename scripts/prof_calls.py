#!/usr/bin/env python3
"""Per-call durations and grid sizes of the kernels matching a name filter in one steady step of a
rocprofv3 kernel trace (kernel_trace.csv): usage prof_calls.py trace.csv filter [marker] [skip]"""
import csv, re, sys

path, filt = sys.argv[1], sys.argv[2]
marker = sys.argv[3] if len(sys.argv) > 3 else "sgd_kernel"
skip = int(sys.argv[4]) if len(sys.argv) > 4 else 4
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
marks = [r for r in rows if marker in r["Kernel_Name"]]
t0, t1 = int(marks[skip - 1]["End_Timestamp"]), int(marks[skip]["End_Timestamp"])
gk = next((k for k in rows[0] if k.lower().startswith("grid_size_x") or k == "Grid_Size_X" or k == "Grid_Size"), None)
for r in rows:
    if t0 < int(r["Start_Timestamp"]) <= t1 and filt in r["Kernel_Name"]:
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        print(f"{us:8.1f} us  grid {r.get(gk, '?'):>9}  {re.sub(r'[(].*', '', r['Kernel_Name'])[:90]}")
