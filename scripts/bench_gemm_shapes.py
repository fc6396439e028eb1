#!/usr/bin/env python3
"""Dense NT GEMM at the implicit-GEMM sizes of ResNet-50's convolutions
(M = N*OH*OW, N = Cout, K = R*S*Cin): 128-tile igemm vs the 256-tile LDS-DMA
kernel vs hipBLASLt -- tells whether a conv loader on the 256 structure pays."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from distributed_pytorch_example_amd.ops._ext import ext  # noqa: E402

C = ext()
dev = "cuda"
SHAPES = [(256 * 56 * 56, 64, 576), (256 * 28 * 28, 128, 1152), (256 * 14 * 14, 256, 2304), (256 * 7 * 7, 512, 4608),
          (256 * 56 * 56, 256, 64), (256 * 28 * 28, 512, 128), (256 * 14 * 14, 1024, 256), (256 * 14 * 14, 256, 1024)]
if len(sys.argv) > 1 and sys.argv[1] == "square":
    SHAPES = [(4096, 4096, 4096), (8192, 8192, 8192), (8192, 8192, 1024), (16384, 4096, 4096)]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


C.set_gemm_backend(1)
for M, N, K in SHAPES:
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
    fl = 2.0 * M * N * K
    res = {"M": M, "N": N, "K": K}
    for name, mode in (("igemm128", 1), ("gemm256", 2)):
        C.set_gemm256_mode(mode)
        res[name + "_TF"] = round(fl / timeit(lambda: C.linear_fwd(x, w, None, 0, False)) / 1e12, 1)
    C.set_gemm256_mode(0)
    res["hipblaslt_TF"] = round(fl / timeit(lambda: x @ w.t()) / 1e12, 1)
    print(json.dumps(res), flush=True)
