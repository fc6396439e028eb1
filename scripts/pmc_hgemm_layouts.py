#!/usr/bin/env python3
"""One 8192^3 GEMM per operand layout (NT, NN, TN; 256x256 tile, no split), a few calls each -- the
workload for a rocprofv3 --pmc pass comparing the layouts' LDS behaviour (scripts/gpu_pmc_hgemm.sh)."""
import sys

import torch

sys.path.insert(0, ".")
from distributed_pytorch_example_amd.ops._ext import ext  # noqa: E402

C = ext()
n = 8192
g = torch.Generator(device="cuda").manual_seed(0)
A = torch.randn(n, n, device="cuda", generator=g).bfloat16()
B = torch.randn(n, n, device="cuda", generator=g).bfloat16()
out = torch.empty(n, n, device="cuda")
for ak, bk in ((True, True), (True, False), (False, False)):
    for _ in range(3):
        C.hgemm(A, B, out, n, n, n, n, n, n, ak, bk, 1, 0, None, None, None, None, 1.0, 0, 1)
torch.cuda.synchronize()
print("done")
