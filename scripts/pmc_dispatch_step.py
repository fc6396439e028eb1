#!/usr/bin/env python3
"""One steady step of a bench run, dispatch by dispatch, with HBM bytes and MFMA busy (two rocprofv3 --pmc passes,
scripts/gpu_pmc_steady.sh layout): the measured side of the per-kernel "compulsory vs measured bytes" table
(docs/perf_notes.md, round 6).  Dispatches of the two passes are aligned by their order inside the step.

usage: pmc_dispatch_step.py <pass-a dir> <pass-b dir> [marker=sgd_kernel] [min_us=20]
rd MB = 2 x FETCH_SIZE (gfx950 reports half the bytes of wide coalesced reads), wr MB = WRITE_SIZE."""
import collections
import csv
import glob
import re
import sys


def load(root):
    cnt = collections.defaultdict(dict)
    meta = {}
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            cnt[d][r["Counter_Name"]] = cnt[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            meta.setdefault(d, (r.get("Kernel_Name", "?"), r.get("Grid_Size", "?")))
    times = {}
    for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            times[d] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
            meta.setdefault(d, (r.get("Kernel_Name", "?"), r.get("Grid_Size", "?")))
    ids = sorted(d for d in times)
    return ids, cnt, meta, times


def step(ids, meta, marker):
    marks = [i for i, d in enumerate(ids) if marker in meta[d][0]]
    a, b = marks[-2], marks[-1]
    return ids[a + 1: b + 1]


marker = sys.argv[3] if len(sys.argv) > 3 else "sgd_kernel"
min_us = float(sys.argv[4]) if len(sys.argv) > 4 else 20.0
ia, ca, ma, ta = load(sys.argv[1])
ib, cb, mb, tb = load(sys.argv[2])
sa, sb = step(ia, ma, marker), step(ib, mb, marker)
if len(sa) != len(sb):
    print(f"# warning: step lengths differ ({len(sa)} vs {len(sb)}); write bytes aligned by order anyway")
print(f"{'#':>4} {'us':>8} {'MFMA%':>6} {'rd MB':>8} {'wr MB':>8} {'TB/s':>6}  grid  kernel")
for n, d in enumerate(sa):
    t0, t1 = ta[d]
    us = (t1 - t0) / 1e3
    if us < min_us:
        continue
    rd = 2.0 * ca[d].get("FETCH_SIZE", 0.0) * 1024 / 1e6
    wr = cb[sb[n]].get("WRITE_SIZE", 0.0) * 1024 / 1e6 if n < len(sb) else 0.0
    mf = 100.0 * ca[d].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (us * 1e-6 * 2.4e9 * 1024) if us > 0 else 0.0
    name = re.sub(r"\(.*", "", ma[d][0])[:80]
    print(f"{n:4d} {us:8.1f} {mf:6.1f} {rd:8.1f} {wr:8.1f} {(rd + wr) / us:6.2f}  {ma[d][1]:>8}  {name}")
