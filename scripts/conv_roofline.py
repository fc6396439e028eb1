#!/usr/bin/env python3
"""Attribute igemm dispatches of ONE ResNet-50 training step (batch B) to conv
layers and passes, and report achieved TF/s and minimum-traffic GB/s."""
import csv, sys
from collections import defaultdict
trace, B = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 256
rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
# last step = dispatches after the second-to-last sgd_kernel
idx = [i for i, r in enumerate(rows) if "sgd_kernel" in r["Kernel_Name"]]
step = rows[idx[-2] + 1: idx[-1] + 1]
ig = [r for r in step if "igemm_kernel" in r["Kernel_Name"]]
# conv list in forward order: (name, Cin, Cout, k, stride, Hin)
convs = [("stem", 8, 64, 7, 2, 224)]
H = 56; inp = 64
for li, (n, planes) in enumerate(zip((3, 4, 6, 3), (64, 128, 256, 512))):
    for j in range(n):
        s = 2 if (j == 0 and li > 0) else 1
        blk = f"L{li+1}.{j}"
        if j == 0: convs.append((blk + ".down", inp, planes * 4, 1, s, H))
        convs.append((blk + ".c1", inp, planes, 1, 1, H))
        convs.append((blk + ".c2", planes, planes, 3, s, H))
        Ho = H // s
        convs.append((blk + ".c3", planes, planes * 4, 1, 1, Ho))
        inp = planes * 4; H = Ho
fwd = ig[:len(convs)]
# backward order per block (reverse): c3 wgrad, c3 dgrad, c2 wgrad, c2 dgrad, c1 wgrad, [down wgrad, down dgrad], c1 dgrad
bwd_names = []
blocks = {}
for c in convs[1:]:
    blocks.setdefault(c[0].rsplit(".", 1)[0], {})[c[0].rsplit(".", 1)[1]] = c
for blk in reversed(list(blocks)):
    b = blocks[blk]
    seq = [("c3", "wgrad"), ("c3", "dgrad"), ("c2", "wgrad"), ("c2", "dgrad"), ("c1", "wgrad")]
    if "down" in b: seq += [("down", "wgrad"), ("down", "dgrad")]
    seq += [("c1", "dgrad")]
    bwd_names += [(b[c], p) for c, p in seq]
bwd_names += [(convs[0], "wgrad")]
bwd = ig[len(convs) + 3:]  # skip fc fwd, fc dgrad, fc wgrad
assert len(bwd) >= len(bwd_names), (len(bwd), len(bwd_names))
def info(c):
    name, ci, co, k, s, h = c
    ho = h // s if not name.startswith("stem") else 112
    M = B * ho * ho
    flop = 2 * M * co * k * k * ci
    return M, ho, flop
tot = defaultdict(float)
print(f"{'layer':14s} {'pass':6s} {'tile':>14s} {'us':>8s} {'TF/s':>7s} {'GB/s':>7s}")
for c, p, r in [(c, "fwd", r) for c, r in zip(convs, fwd)] + [(c, p, r) for (c, p), r in zip(bwd_names, bwd)]:
    name, ci, co, k, s, h = c
    M, ho, flop = info(c)
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    inb = B * h * h * ci * 2; outb = M * co * 2; wb = co * k * k * ci * 2
    byts = {"fwd": inb + outb + wb, "dgrad": outb + inb + wb, "wgrad": inb + outb + wb * 2}[p]
    tile = r["Kernel_Name"].split("<")[1].split(">")[0]
    tot[p] += us
    print(f"{name:14s} {p:6s} {tile:>14s} {us:8.1f} {flop/us/1e6:7.1f} {byts/us/1e3:7.1f}")
print({k: round(v / 1e3, 2) for k, v in tot.items()}, "ms")
