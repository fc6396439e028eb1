#!/usr/bin/env python3
"""Run one hgemm configuration a few times (for rocprofv3 --pmc / kernel-trace passes).
usage: hgemm_one.py LAYOUT M N K [cfg] [reps]   LAYOUT in fwd|dgrad|wgrad"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_example_amd.ops._ext import ext  # noqa: E402

C = ext()
lay, M, N, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
cfg = int(sys.argv[5]) if len(sys.argv) > 5 else 0
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 5
dev = "cuda"
if lay == "fwd":
    A, B, lda, ldb, ak, bk = torch.randn(M, K, device=dev).bfloat16(), torch.randn(N, K, device=dev).bfloat16(), K, K, True, True
elif lay == "dgrad":
    A, B, lda, ldb, ak, bk = torch.randn(M, K, device=dev).bfloat16(), torch.randn(K, N, device=dev).bfloat16(), K, N, True, False
else:
    A, B, lda, ldb, ak, bk = torch.randn(K, M, device=dev).bfloat16(), torch.randn(K, N, device=dev).bfloat16(), M, N, False, False
out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
for _ in range(reps):
    C.hgemm(A, B, out, M, N, K, lda, ldb, N, ak, bk, 0, 0, None, None, None, None, 1.0, cfg, 1)
torch.cuda.synchronize()
print("done", lay, M, N, K, cfg)
