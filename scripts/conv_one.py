#!/usr/bin/env python3
"""Run ONE conv pass shape repeatedly (for rocprofv3 PMC collection)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sys, torch
from distributed_pytorch_example_amd.ops import ext
C = ext()
ci, co, k, s, h, B = [int(v) for v in sys.argv[1:7]]
ps = sys.argv[7] if len(sys.argv) > 7 else "fwd"
reps = int(sys.argv[8]) if len(sys.argv) > 8 else 20
p = k // 2; ho = (h + 2 * p - k) // s + 1
x = torch.randn(B, h, h, ci, device="cuda").to(torch.bfloat16)
w = (torch.randn(co, k, k, ci, device="cuda") / (k * k * ci) ** 0.5).to(torch.bfloat16)
dy = torch.randn(B, ho, ho, co, device="cuda").to(torch.bfloat16)
dw = torch.zeros(co, k, k, ci, device="cuda")
for _ in range(reps):
    if ps == "fwd": C.conv_fwd(x, w, [s, s], [p, p], [1, 1], False, None)
    elif ps == "dgrad": C.conv_dgrad(dy, w, list(x.shape), [s, s], [p, p], [1, 1], None)
    else: C.conv_wgrad(dy, x, dw, [s, s], [p, p], [1, 1], 1.0)
torch.cuda.synchronize()
