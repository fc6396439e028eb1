#!/usr/bin/env python3
"""Strided 1x1 (downsample) conv forwards with BN sums at batch 512: the persistent GEMM's implicit-im2col
route vs the implicit-GEMM kernel (set_hgemm_conv).  One JSON line per shape and arm."""
import json
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "scripts")
from distributed_pytorch_example_amd.ops._ext import ext  # noqa: E402
from bench_hgemm import timeit  # noqa: E402

C = ext()
for H, Ci, Co in ((56, 256, 512), (28, 512, 1024), (14, 1024, 2048)):
    x = torch.randn(512, H, H, Ci, device="cuda").bfloat16()
    w = (torch.randn(Co, 1, 1, Ci, device="cuda") / Ci ** 0.5).bfloat16()
    fl = 2.0 * 512 * (H // 2) ** 2 * Ci * Co
    for on in (True, False):
        C.set_hgemm_conv(on)
        t = timeit(lambda: C.conv_fwd(x, w, [2, 2], [0, 0], [1, 1], True, None))
        print(json.dumps({"H": H, "Cin": Ci, "Cout": Co, "hgemm": on, "us": round(t, 1), "TF": round(fl / t / 1e6, 1)}),
              flush=True)
C.set_hgemm_conv(True)
