#!/usr/bin/env python3
"""Average rocprofv3 --pmc counters per kernel over every *counter_collection.csv under a dir."""
import collections, csv, glob, sys

root = sys.argv[1]
title = sys.argv[2] if len(sys.argv) > 2 else root
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", "?")
        if "dpe::" not in name:
            continue
        key = name.split("(")[0][:90]
        acc[key][row["Counter_Name"]].append(float(row["Counter_Value"]))
print(title)
for k, cs in acc.items():
    print(k)
    for c in sorted(cs):
        v = cs[c]
        print(f"   {c:28s} {sum(v) / len(v):.4g}  (n={len(v)})")
