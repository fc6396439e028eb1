#!/usr/bin/env python3
"""Driver for scripts/gpu_pmc_kernels.sh: the layer-2 3x3 data grad + BN partials, batch 512, on the 128x128
LDS-DMA tile -- "phase": the strided conv's 4 parity sub-GEMMs (dx 56^2), "s1": the stride-1 conv (dx 28^2)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_pytorch_example_amd.ops import ext  # noqa: E402

C = ext()
mode = sys.argv[1]
B, ci, co = 512, 128, 128
h = 56 if mode == "phase" else 28
st = 2 if mode == "phase" else 1
ho = h // st
w = (torch.randn(co, 3, 3, ci, device="cuda") / (9 * ci) ** 0.5).to(torch.bfloat16)
dy = torch.randn(B, ho, ho, co, device="cuda").to(torch.bfloat16)
hh = torch.randn(B, h, h, ci, device="cuda").to(torch.bfloat16)
coef = torch.stack([torch.rand(ci, device="cuda") + 0.5, torch.randn(ci, device="cuda") * 0.1,
                    torch.randn(ci, device="cuda") * 0.1, torch.rand(ci, device="cuda") + 0.5]).contiguous()
C.set_conv_tile(1)
for _ in range(10):
    C.conv_dgrad_bn(dy, w, [B, h, h, ci], [st, st], [1, 1], [1, 1], None, hh, coef)
torch.cuda.synchronize()
