#!/usr/bin/env python3
"""ResNet-50 1x1 stride-1 convs at batch 512: the conv paths (with their BN epilogues) vs the
persistent hgemm on the same GEMM (no BN epilogue) -- is moving them onto hgemm worth a BN epilogue?"""
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
for H, Ci, Co in [(56, 256, 64), (56, 64, 256), (28, 512, 128), (28, 128, 512), (14, 1024, 256), (14, 256, 1024),
                  (7, 2048, 512), (7, 512, 2048)]:
    B = 512
    M = B * H * H
    x = torch.randn(B, H, H, Ci, device="cuda").to(bf)
    w = (torch.randn(Co, 1, 1, Ci, device="cuda") / Ci ** 0.5).to(bf)
    dy = torch.randn(B, H, H, Co, device="cuda").to(bf)
    coef = torch.stack([torch.rand(Ci, device="cuda") + .5, torch.randn(Ci, device="cuda"),
                        torch.randn(Ci, device="cuda"), torch.rand(Ci, device="cuda") + .5]).contiguous()
    fl = 2 * M * Ci * Co
    t_conv = timeit(lambda: C.conv_fwd(x, w, [1, 1], [0, 0], [1, 1], True, None))
    t_lin = timeit(lambda: C.linear_fwd(x.view(M, Ci), w.view(Co, Ci)))
    t_dg = timeit(lambda: C.conv_dgrad_bn(dy, w, [B, H, H, Ci], [1, 1], [0, 0], [1, 1], None, x, coef))
    t_ldg = timeit(lambda: C.linear_dgrad(dy.view(M, Co), w.view(Co, Ci)))
    print(json.dumps({"H": H, "Cin": Ci, "Cout": Co, "conv_fwd_us": round(t_conv, 1), "hgemm_fwd_us": round(t_lin, 1),
                      "conv_fwd_TF": round(fl / t_conv / 1e6), "hgemm_fwd_TF": round(fl / t_lin / 1e6),
                      "conv_dgrad_bn_us": round(t_dg, 1), "hgemm_dgrad_us": round(t_ldg, 1)}), flush=True)
    del x, w, dy
    torch.cuda.empty_cache()
