#!/usr/bin/env python3
"""Interleaved A/B of hgemm arms (cdna_hip_programming.md §5.4 rule 24: N variants x M rounds in
ONE process, report median and min).  usage:
    ab_hgemm.py [--rounds 7] [--iters 20] [--shapes sq8192.fwd,qkv.fwd,...] --arm name:cfg,splits,group_m ...
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_example_amd.ops._ext import ext  # noqa: E402

C = ext()
dev = "cuda"
T = 8192
SH = {
    "qkv.fwd": (T, 2304, 768, "fwd"), "proj.fwd": (T, 768, 768, "fwd"), "fc.fwd": (T, 3072, 768, "fwd"),
    "mproj.fwd": (T, 768, 3072, "fwd"), "lmhead.fwd": (T, 50304, 768, "fwd"),
    "qkv.dgrad": (T, 768, 2304, "dgrad"), "fc.dgrad": (T, 768, 3072, "dgrad"), "mproj.dgrad": (T, 3072, 768, "dgrad"),
    "lmhead.dgrad": (T, 768, 50304, "dgrad"),
    "qkv.wgrad": (2304, 768, T, "wgrad"), "fc.wgrad": (3072, 768, T, "wgrad"), "lmhead.wgrad": (50304, 768, T, "wgrad"),
}
for n in (4096, 8192):
    for lay in ("fwd", "dgrad", "wgrad"):
        SH[f"sq{n}.{lay}"] = (n, n, n, lay)


def operands(M, N, K, lay):
    g = torch.Generator(device=dev).manual_seed(0)
    if lay == "fwd":
        return (torch.randn(M, K, device=dev, generator=g).bfloat16(), torch.randn(N, K, device=dev, generator=g).bfloat16(),
                K, K, True, True)
    if lay == "dgrad":
        return (torch.randn(M, K, device=dev, generator=g).bfloat16(), torch.randn(K, N, device=dev, generator=g).bfloat16(),
                K, N, True, False)
    return (torch.randn(K, M, device=dev, generator=g).bfloat16(), torch.randn(K, N, device=dev, generator=g).bfloat16(),
            M, N, False, False)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--shapes", default="sq8192.fwd,sq8192.dgrad,sq8192.wgrad,qkv.fwd,fc.dgrad,lmhead.fwd")
    ap.add_argument("--arm", action="append", default=[])
    a = ap.parse_args()
    arms = []
    for spec in a.arm or ["plan:-1,-1,0"]:
        name, v = spec.split(":")
        cfg, sp, gm = (int(x) for x in v.split(","))
        arms.append((name, cfg, sp, gm))
    for shp in a.shapes.split(","):
        M, N, K, lay = SH[shp]
        A, B, lda, ldb, ak, bk = operands(M, N, K, lay)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        times = {n: [] for n, *_ in arms}
        for r in range(a.rounds + 1):
            for name, cfg, sp, gm in arms:
                def f():
                    C.hgemm(A, B, out, M, N, K, lda, ldb, N, ak, bk, 0, 0, None, None, None, None, 1.0, cfg, sp, gm)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                f()
                s.record()
                for _ in range(a.iters):
                    f()
                e.record()
                torch.cuda.synchronize()
                if r > 0:  # round 0 = warm-up
                    times[name].append(s.elapsed_time(e) * 1e3 / a.iters)
        row = {"shape": shp}
        for n, ts in times.items():
            row[n] = {"med_TF": round(fl / statistics.median(ts) / 1e6, 1), "best_TF": round(fl / min(ts) / 1e6, 1)}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
