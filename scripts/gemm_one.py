#!/usr/bin/env python3
"""Run one GEMM shape repeatedly (for rocprofv3 PMC collection).
usage: gemm_one.py kind M N K iters [mode]   kind in fwd|dgrad|wgrad|torch ; mode 0 auto / 1 igemm / 2 force gemm256"""
import sys

import torch

sys.path.insert(0, ".")
from distributed_pytorch_example_amd.ops._ext import ext  # noqa: E402

kind, M, N, K, iters = sys.argv[1], *map(int, sys.argv[2:6])
mode = int(sys.argv[6]) if len(sys.argv) > 6 else 0
C = ext()
C.set_gemm256_mode(mode)
dev = "cuda"
x = torch.randn(M, K, device=dev).to(torch.bfloat16)
w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
dw = torch.zeros(N, K, device=dev)
for _ in range(iters):
    if kind == "fwd":
        C.linear_fwd(x, w, None, 0, False)
    elif kind == "torch":
        x @ w.t()
    elif kind == "dgrad":
        C.linear_dgrad(x[:, :N].contiguous() if K >= N else torch.randn(M, N, device=dev).to(torch.bfloat16), w)
    else:
        C.linear_wgrad(torch.randn(M, N, device=dev).to(torch.bfloat16), x, dw, 1.0)
torch.cuda.synchronize()
