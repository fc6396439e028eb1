#!/usr/bin/env python3
"""8192^3 (and 4096^3) persistent-GEMM throughput per operand layout (256x256 tile, no split): the
per-CU rates the planner's cost model uses (bindings/gemm.cpp layout_rate).  One JSON line each."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_example_amd.ops._ext import ext  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_hgemm import timeit  # noqa: E402

C = ext()
for n in (8192, 4096):
    g = torch.Generator(device="cuda").manual_seed(0)
    A = torch.randn(n, n, device="cuda", generator=g).bfloat16()
    B = torch.randn(n, n, device="cuda", generator=g).bfloat16()
    out = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    for name, ak, bk in (("NT", True, True), ("NN", True, False), ("TN", False, False)):
        us = timeit(lambda: C.hgemm(A, B, out, n, n, n, n, n, n, ak, bk, 0, 0, None, None, None, None, 1.0, 0, 1))
        print(json.dumps({"n": n, "layout": name, "us": round(us, 1), "tflops": round(2 * n ** 3 / us / 1e6, 1)}), flush=True)
