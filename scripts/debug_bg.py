#!/usr/bin/env python3
"""Structured probe of the TN weight-grad GEMM's fused bias gradient (hgemm BG): A = dy^T [K][M]
filled with 1, with its row index m, with its k index, and random; prints expected vs got rows."""
import sys

import torch

sys.path.insert(0, ".")
from distributed_pytorch_example_amd.ops._ext import ext  # noqa: E402

C = ext()
dev = "cuda"
for M, N, K in ((256, 256, 64), (256, 256, 128), (520, 776, 832)):
    for name, fill in (("ones", lambda k, m: torch.ones(k, m)), ("m", lambda k, m: torch.arange(m).float().expand(k, m) % 64),
                       ("k", lambda k, m: (torch.arange(k).float()[:, None] % 64).expand(k, m)),
                       ("rand", lambda k, m: torch.randn(k, m))):
        A = fill(K, M).contiguous().to(dev).bfloat16()
        B = torch.randn(K, N, device=dev).bfloat16()
        out = torch.zeros(M, N, device=dev)
        db = torch.zeros(M, device=dev)
        C.hgemm(A, B, out, M, N, K, M, N, N, False, False, 2, 0, None, None, None, None, 1.0, 0, 1, 0, db)
        torch.cuda.synchronize()
        want = A.float().sum(0)
        err = ((db - want).norm() / want.norm().clamp_min(1e-9)).item()
        print(f"M{M} N{N} K{K} {name:5s} err {err:.3e}  got[:20] {db[:20].tolist()}  want[:20] {want[:20].tolist()}", flush=True)
        if name == "rand":
            bad = ((db - want).abs() > 1e-2 * want.abs().max()).nonzero().flatten()
            print(f"   bad rows: {bad.numel()} first {bad[:40].tolist()}; ratio got/want rows 0..8 "
                  f"{(db[:8] / want[:8]).tolist()}", flush=True)
