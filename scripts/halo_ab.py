#!/usr/bin/env python3
"""Layer-1 3x3 conv (64 -> 64 @ 56x56, batch 512): halo-tiled kernel vs LDS-DMA tile, forward /
data grad / data grad with the BN-backward epilogue (set_conv3_halo toggled in-process)."""
import os, sys, statistics
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_pytorch_example_amd.ops import ext
C = ext()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
x = torch.randn(B, 56, 56, 64, device="cuda").to(torch.bfloat16)
w = (torch.randn(64, 3, 3, 64, device="cuda") / 24).to(torch.bfloat16)
dy = torch.randn(B, 56, 56, 64, device="cuda").to(torch.bfloat16)
h = torch.randn(B, 56, 56, 64, device="cuda").to(torch.bfloat16)
coef = torch.cat([torch.rand(64) + 0.5, torch.randn(64), torch.randn(64) * 0.1, torch.rand(64) + 0.5]).cuda()
z = [1, 1], [1, 1], [1, 1]
ops = {"fwd": lambda: C.conv_fwd(x, w, *z, True, None),
       "dgrad": lambda: C.conv_dgrad(dy, w, [B, 56, 56, 64], *z, None),
       "dgrad_bn": lambda: C.conv_dgrad_bn(dy, w, [B, 56, 56, 64], *z, None, h, coef)}
flops = 2 * B * 56 * 56 * 64 * 576
for rep in range(2):
    for on in (False, True):
        C.set_conv3_halo(on)
        for name, fn in ops.items():
            for _ in range(3):
                fn()
            ts = []
            for _ in range(15):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(); fn(); b.record(); b.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
            t = statistics.median(ts)
            print(f"halo={int(on)} {name:9s} {t:8.1f} us  {flops / t / 1e6:7.1f} TF/s", flush=True)
