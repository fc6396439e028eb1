#!/usr/bin/env python3
"""Interleaved A/B of the s2d stem weight grad at batch 512 (16 ch 112x112 -> 64, 4x4 pad 2-2-1-1):
row-walking kernel (set_stem_kernel on) vs the im2col weight-grad tile; CUDA-event medians, TF/s."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import statistics
import torch
from distributed_pytorch_example_amd.ops import ext

C = ext()
B, H = int(sys.argv[1]) if len(sys.argv) > 1 else 512, 112
x = torch.randn(B, H, H, 16, device="cuda").to(torch.bfloat16)
dy = torch.randn(B, H, H, 64, device="cuda").to(torch.bfloat16)
dw = torch.zeros(64, 4, 4, 16, device="cuda")
res = {True: [], False: []}
out = {}
for rep in range(14):
    for on in (True, False):
        C.set_stem_kernel(on)
        dw.zero_()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        C.conv_wgrad(dy, x, dw, [1, 1], [2, 2], [1, 1], 1.0)
        b.record()
        b.synchronize()
        if rep >= 4:
            res[on].append(a.elapsed_time(b) * 1e3)
        out[on] = dw.clone()
C.set_stem_kernel(True)
fl = 2.0 * B * H * H * 64 * 256
for on in (True, False):
    m = statistics.median(res[on])
    print(f"{'row kernel' if on else 'im2col tile'}: {m:7.1f} us  {fl / m / 1e6:6.1f} TF", flush=True)
print(f"rel diff {((out[True] - out[False]).norm() / out[False].norm()).item():.2e}")
