#!/usr/bin/env python3
"""GPT-2 weight-gradient GEMMs (dW[N,K] += dY[M,N]^T X[M,K], M = tokens) per arm:
hipBLASLt (addmm into fp32), the autotuned linear_wgrad, and the LDS-DMA
split-K weight-grad kernel reached as a 1x1 convolution over a [1, M, 1, C] image.
Run with DPE_WGRAD_DMA=2 so the 1x1 conv arm takes the DMA kernel.
usage: DPE_WGRAD_DMA=2 python scripts/bench_linear_wgrad.py [tokens]"""
import json
import sys

import torch

sys.path.insert(0, ".")
from distributed_pytorch_example_amd.ops._ext import ext  # noqa: E402


def t_ms(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


C = ext()
M = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
dev = "cuda"
for (N, K) in [(3072, 768), (768, 3072), (2304, 768), (768, 768)]:
    dy = (torch.randn(M, N, device=dev) * 0.1).to(torch.bfloat16)
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    ref = dy.float().t() @ x.float()
    dw_b, dw_l, dw_c = (torch.zeros(N, K, device=dev) for _ in range(3))
    fl = 2.0 * M * N * K
    tb = t_ms(lambda: torch.addmm(dw_b, dy.t(), x, out_dtype=torch.float32))
    tl = t_ms(lambda: C.linear_wgrad(dy, x, dw_l, 1.0))
    dy4, x4, dw4 = dy.view(1, M, 1, N), x.view(1, M, 1, K), dw_c.view(N, 1, 1, K)
    tc = t_ms(lambda: C.conv_wgrad(dy4, x4, dw4, [1, 1], [0, 0], [1, 1], 1.0))
    # numerics: one fresh accumulation per arm
    dw_l.zero_(); C.linear_wgrad(dy, x, dw_l, 1.0)
    dw_c.zero_(); C.conv_wgrad(dy4, x4, dw4, [1, 1], [0, 0], [1, 1], 1.0)
    torch.cuda.synchronize()
    err_l = ((dw_l - ref).abs().max() / ref.abs().max()).item()
    err_c = ((dw_c - ref).abs().max() / ref.abs().max()).item()
    print(json.dumps({"M": M, "N": N, "K": K, "hipblaslt_us": round(tb * 1e3, 1), "linear_wgrad_us": round(tl * 1e3, 1),
                      "conv1x1_dma_us": round(tc * 1e3, 1), "hipblaslt_TF": round(fl / tb / 1e9, 1),
                      "conv1x1_dma_TF": round(fl / tc / 1e9, 1), "relerr_linear": err_l, "relerr_conv": err_c}), flush=True)
