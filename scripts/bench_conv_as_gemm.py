#!/usr/bin/env python3
"""Ceiling check: the persistent GEMM (hgemm) on dense GEMMs of the ResNet-50 3x3-conv shapes
(M = N*OH*OW, N = Cout, K = 9*Cin) vs our implicit-GEMM conv on the real conv (batch 512)."""
import json, os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_pytorch_example_amd.ops import ext


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


C = ext()
bf = torch.bfloat16
for H, Ci, Co, s in [(28, 128, 128, 1), (14, 256, 256, 1), (7, 512, 512, 1), (56, 128, 128, 2), (28, 256, 256, 2), (14, 512, 512, 2)]:
    B = 512
    OH = H if s == 1 else H // 2
    M, K = B * OH * OH, 9 * Ci
    a = torch.randn(M, K, device="cuda").to(bf)
    w = (torch.randn(Co, K, device="cuda") / K ** 0.5).to(bf)
    x = torch.randn(B, H, H, Ci, device="cuda").to(bf)
    w4 = w.view(Co, 3, 3, Ci).contiguous()
    fl = 2 * M * K * Co
    t_g = timeit(lambda: C.linear_fwd(a, w))
    t_c = timeit(lambda: C.conv_fwd(x, w4, [s, s], [1, 1], [1, 1], True, None))
    print(json.dumps({"H": H, "Cin": Ci, "Cout": Co, "stride": s, "M": M, "K": K, "hgemm_us": round(t_g, 1),
                      "hgemm_TF": round(fl / t_g / 1e6), "conv_us": round(t_c, 1), "conv_TF": round(fl / t_c / 1e6)}), flush=True)
    del a, w, x, w4
    torch.cuda.empty_cache()
