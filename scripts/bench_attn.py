#!/usr/bin/env python3
"""Attention kernels at the GPT-2-small training shape (B=8, T=1024, H=12, D=64, causal),
timed with HIP events.

usage: bench_attn.py [--reps 50] [--B 8 --T 1024 --H 12]
(A/B against another build: run it again with DPE_EXT_SO=<other _C.so>, alternating processes --
two pybind builds of the module cannot share one process.)
Prints one JSON line per (build, pass): us per call and TFLOP/s (causal FLOPs:
fwd 2*B*H*T^2*D, bwd dK/dV + dQ 2.5x that, the delta pass included in the bwd time).
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--H", type=int, default=12)
    a = ap.parse_args()
    from distributed_pytorch_example_amd.ops import ext

    builds = [(os.environ.get("DPE_EXT_SO", "cur"), ext())]
    B, T, H, D = a.B, a.T, a.H, 64
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    qkv = torch.randn(B, T, 3, H, D, device=dev).to(torch.bfloat16)
    do = torch.randn(B, T, H, D, device=dev).to(torch.bfloat16)
    scale = 1.0 / math.sqrt(D)
    fl_f = 2.0 * B * H * T * T * D  # causal: half of 4*B*H*T^2*D
    res = {n: {"fwd": [], "bwd": []} for n, _ in builds}
    for n, C in builds:  # warm-up + outputs for a cross-build check
        out, lse = C.attn_fwd(qkv, H, scale, True)
        dq = C.attn_bwd(qkv, out, do, lse, H, scale, True)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for _ in range(5):
        for n, C in builds:
            out, lse = C.attn_fwd(qkv, H, scale, True)
            ev[0].record()
            for _ in range(a.reps):
                C.attn_fwd(qkv, H, scale, True)
            ev[1].record()
            for _ in range(a.reps):
                C.attn_bwd(qkv, out, do, lse, H, scale, True)
            ev[2].record()
            torch.cuda.synchronize()
            res[n]["fwd"].append(ev[0].elapsed_time(ev[1]) * 1e3 / a.reps)
            res[n]["bwd"].append(ev[1].elapsed_time(ev[2]) * 1e3 / a.reps)
    for n, _ in builds:
        f, b = min(res[n]["fwd"]), min(res[n]["bwd"])
        print(json.dumps({"build": n, "shape": [B, T, H, D], "fwd_us": round(f, 2), "fwd_tflops": round(fl_f / f / 1e6, 1),
                          "bwd_us": round(b, 2), "bwd_tflops": round(2.5 * fl_f / b / 1e6, 1)}))


if __name__ == "__main__":
    main()
