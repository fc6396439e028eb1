#!/usr/bin/env python3
"""Per-shape timing of the ResNet-50 convolutions (batch B): our gfx950
implicit-GEMM kernels vs MIOpen (torch channels_last bf16) for fwd / dgrad /
wgrad.  Random non-zero data; CUDA-event timing, median of N reps."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import argparse
import json
import statistics

import torch
import torch.nn.functional as F

from distributed_pytorch_example_amd.ops import ext

SHAPES = [  # (Cin, Cout, k, stride, Hin, count in ResNet-50)
    (8, 64, 7, 2, 224, 1),
    (64, 64, 1, 1, 56, 1), (64, 64, 3, 1, 56, 3), (64, 256, 1, 1, 56, 4), (256, 64, 1, 1, 56, 2),
    (256, 128, 1, 1, 56, 1), (128, 128, 3, 2, 56, 1), (256, 512, 1, 2, 56, 1), (128, 512, 1, 1, 28, 4),
    (512, 128, 1, 1, 28, 3), (128, 128, 3, 1, 28, 3), (512, 256, 1, 1, 28, 1), (256, 256, 3, 2, 28, 1),
    (512, 1024, 1, 2, 28, 1), (256, 1024, 1, 1, 14, 6), (1024, 256, 1, 1, 14, 5), (256, 256, 3, 1, 14, 5),
    (1024, 512, 1, 1, 14, 1), (512, 512, 3, 2, 14, 1), (1024, 2048, 1, 2, 14, 1), (512, 2048, 1, 1, 7, 3),
    (2048, 512, 1, 1, 7, 2), (512, 512, 3, 1, 7, 2),
]


def timeit(fn, reps):
    ts = []
    for _ in range(3):
        fn()
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--miopen", type=int, default=1)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    C = ext()
    torch.backends.cudnn.benchmark = True
    B = args.batch
    tot = {"ours": {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}, "miopen": {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}}
    rows = []
    print(f"{'shape':28s} {'pass':6s} {'ours us':>9s} {'TF/s':>7s} {'miopen us':>10s} {'ratio':>6s}")
    for ci, co, k, s, h, cnt in SHAPES:
        p = k // 2
        ho = (h + 2 * p - k) // s + 1
        x = torch.randn(B, h, h, ci, device="cuda").to(torch.bfloat16)
        if ci == 8:
            x[..., 3:] = 0
        w = (torch.randn(co, k, k, ci, device="cuda") / (k * k * ci) ** 0.5).to(torch.bfloat16)
        dy = torch.randn(B, ho, ho, co, device="cuda").to(torch.bfloat16)
        dw = torch.zeros(co, k, k, ci, device="cuda")
        flop = 2.0 * B * ho * ho * co * k * k * ci
        ours = {
            "fwd": lambda: C.conv_fwd(x, w, [s, s], [p, p], [1, 1], True, None),
            "dgrad": lambda: C.conv_dgrad(dy, w, list(x.shape), [s, s], [p, p], [1, 1], None),
            "wgrad": lambda: C.conv_wgrad(dy, x, dw, [s, s], [p, p], [1, 1], 1.0),
        }
        xm = x.permute(0, 3, 1, 2)  # NCHW view of NHWC memory = channels_last
        wm = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        dym = dy.permute(0, 3, 1, 2)
        mi = {
            "fwd": lambda: F.conv2d(xm, wm, None, s, p),
            "dgrad": lambda: torch.ops.aten.convolution_backward(dym, xm, wm, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                                                 [True, False, False]),
            "wgrad": lambda: torch.ops.aten.convolution_backward(dym, xm, wm, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                                                 [False, True, False]),
        }
        for ps in ("fwd", "dgrad", "wgrad"):
            if ps == "dgrad" and ci == 8:
                continue
            t_o = timeit(ours[ps], args.reps)
            t_m = timeit(mi[ps], args.reps) if args.miopen else float("nan")
            tot["ours"][ps] += t_o * cnt
            tot["miopen"][ps] += t_m * cnt
            rows.append({"shape": [ci, co, k, s, h], "count": cnt, "pass": ps, "ours_us": t_o, "miopen_us": t_m})
            print(f"{str((ci, co, k, s, h)):28s} {ps:6s} {t_o:9.1f} {flop / t_o / 1e6:7.1f} {t_m:10.1f} {t_m / t_o:6.2f}")
    for who in tot:
        print(who, {k: round(v / 1e3, 3) for k, v in tot[who].items()}, "ms/step total",
              round(sum(tot[who].values()) / 1e3, 3))
    if args.json:
        json.dump({"batch": B, "rows": rows, "totals_ms": {w: {k: v / 1e3 for k, v in d.items()} for w, d in tot.items()}},
                  open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
