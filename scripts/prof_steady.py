#!/usr/bin/env python3
"""Steady-state per-step kernel breakdown from a rocprofv3 kernel trace (kernel_trace.csv or the
default rocpd results .db).

Keeps only kernels launched after the K-th call of a per-step marker kernel
(default: the optimizer kernel, one launch per step), so warm-up and GEMM
autotuning trials are excluded.  usage: prof_steady.py trace.csv [skip_steps] [marker] [topN]
"""
import collections, csv, re, sys

path = sys.argv[1]
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 2
marker = sys.argv[3] if len(sys.argv) > 3 else "adam_kernel"
top = int(sys.argv[4]) if len(sys.argv) > 4 else 40
if path.endswith(".db"):
    import sqlite3
    q = sqlite3.connect(path).execute("select name, start, end from kernels")
    rows = [{"Kernel_Name": n, "Start_Timestamp": a, "End_Timestamp": b} for n, a, b in q]
else:
    rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [r for r in rows if marker in r["Kernel_Name"]]
t0 = int(marks[skip - 1]["End_Timestamp"])
t1 = int(marks[-1]["End_Timestamp"])
steps = len(marks) - skip
sel = [r for r in rows if t0 < int(r["Start_Timestamp"]) <= t1]
agg = collections.defaultdict(lambda: [0, 0])
for r in sel:
    n = re.sub(r"\(.*", "", r["Kernel_Name"])[:100]
    agg[n][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg[n][1] += 1
busy = sum(v[0] for v in agg.values())
print(f"{steps} steady steps: wall {(t1 - t0) / 1e6 / steps:.3f} ms/step, kernel-busy {busy / 1e6 / steps:.3f} ms/step, "
      f"{len(sel) / steps:.0f} launches/step")
for n, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
    print(f"{t / 1e6 / steps:7.3f} ms/step {100 * t / busy:5.1f}%  calls/step={c / steps:5.1f} avg={t / c / 1e3:8.1f}us  {n}")
