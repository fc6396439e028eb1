#!/usr/bin/env python3
"""Ceiling check for the 3x3-conv weight grads: the persistent GEMM (hgemm, TN layout, planner's tile and
K split) on DENSE operands of the same GEMM shape (M = Cout, N = 9*Cin, K = batch pixels) vs our
im2col LDS-DMA weight-grad kernel on the real conv (batch 512).  Median of CUDA-event timings."""
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
out = []
for H, Ci, Co, s in [(56, 64, 64, 1), (28, 128, 128, 1), (14, 256, 256, 1), (7, 512, 512, 1), (56, 128, 128, 2),
                     (28, 256, 256, 2), (14, 512, 512, 2)]:
    B = 512
    OH = H // s
    K, M, N = B * OH * OH, Co, 9 * Ci
    a = torch.randn(K, M, device="cuda").to(bf)
    b = torch.randn(K, N, device="cuda").to(bf)
    c = torch.zeros(M, N, device="cuda")
    x = torch.randn(B, H, H, Ci, device="cuda").to(bf)
    dy = torch.randn(B, OH, OH, Co, device="cuda").to(bf)
    dw = torch.zeros(Co, 3, 3, Ci, device="cuda")
    flop = 2.0 * M * N * K
    th = timeit(lambda: C.hgemm(a, b, c, M, N, K, M, N, N, False, False, 2))  # HE_ACC_F32
    tc = timeit(lambda: C.conv_wgrad(dy, x, dw, [s, s], [1, 1], [1, 1], 1.0))
    r = {"H": H, "Cin": Ci, "Cout": Co, "stride": s, "M": M, "N": N, "K": K, "plan": C.hgemm_plan(M, N, K, False, False, True, 4),
         "hgemm_us": round(th, 1), "hgemm_TF": round(flop / th / 1e6), "conv_us": round(tc, 1), "conv_TF": round(flop / tc / 1e6)}
    print(json.dumps(r), flush=True)
