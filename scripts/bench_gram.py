#!/usr/bin/env python3
"""Gram pass (bngram.hip) per ResNet-50 bs512 shape: LDS-DMA kernel vs the register-staged one (DPE_GRAM_DMA)."""
import json, os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_pytorch_example_amd.ops._ext import ext

X = ext()


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


for C, HW in [(64, 56), (128, 28), (256, 14), (512, 7)]:
    M = 512 * HW * HW
    if C > 256:
        continue
    x = torch.randn(M, C, device="cuda").bfloat16()
    coef = torch.stack([torch.ones(C, device="cuda"), 0.1 * torch.randn(C, device="cuda"), torch.zeros(C, device="cuda"),
                        torch.ones(C, device="cuda")]).float()
    row = {"C": C, "M": M, "MB": round(M * C * 2 / 1e6, 1)}
    for arm in ("1", "0"):
        os.environ["DPE_GRAM_DMA"] = arm
        t = timeit(lambda: X.bn_gram(x, coef, coef))
        row["dma_us" if arm == "1" else "reg_us"] = round(t, 1)
    print(json.dumps(row), flush=True)
