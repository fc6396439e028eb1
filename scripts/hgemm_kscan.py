#!/usr/bin/env python3
"""Per-unit fixed cost of the persistent GEMM: time t(K) = a + b K at fixed M, N and tile, so the
intercept a (prologue fill + epilogue drain per round of units) can be compared with the K-loop
slope b (MFMA-bound main loop).  One JSON line per (layout, N, cfg, K):

    python scripts/hgemm_kscan.py [dynamic schedule 1|0]
"""
import json
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "scripts")
from distributed_pytorch_example_amd.ops._ext import ext  # noqa: E402
from bench_hgemm import operands, timeit  # noqa: E402

C = ext()
M = 8192
dyn = int(sys.argv[1]) if len(sys.argv) > 1 else 1
C.set_hgemm_dynamic(bool(dyn))
for lay, N, cfgs in (("fwd", 2304, (0, 3)), ("fwd", 768, (1, 3)), ("dgrad", 768, (0, 1)), ("dgrad", 3072, (0, 1))):
    for cfg in cfgs:
        for K in (768, 1536, 3072, 6144):
            A, B, lda, ldb, ak, bk, _ = operands(M, N, K, lay)
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            t = timeit(lambda: C.hgemm(A, B, out, M, N, K, lda, ldb, N, ak, bk, 0, 0, None, None, None, None, 1.0, cfg, 1))
            print(json.dumps({"dyn": dyn, "layout": lay, "M": M, "N": N, "K": K, "cfg": cfg, "us": round(t, 2),
                              "TF": round(2.0 * M * N * K / t / 1e6, 1)}), flush=True)
