#!/usr/bin/env python3
"""Per-tile time of the persistent GEMM vs the number of busy CUs: one 256x256 tile per block (K = 4608, cfg forced
to 256x256 with no K split), tiles 16..512, as N = 256 (M = 256 x tiles: every tile streams its own A rows,
~256 FLOP per HBM byte) and as N = 2048 (8 tile columns share each A row band through L2).  In one round (tiles <= 256) every block
does the same work, so a rising time says the chip runs each CU slower the more of them are busy (clocks /
power or shared L2-MALL-HBM bandwidth) -- why a partly idle last round costs less than its share."""
import json, os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_pytorch_example_amd.ops import ext


def timeit(fn, reps=20):
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
K = 4608
for N in (256, 2048):
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(bf)
    for tiles in (16, 32, 64, 128, 160, 192, 224, 256, 320, 384, 448, 512):
        M = 256 * tiles * 256 // N
        a = torch.randn(M, K, device="cuda").to(bf)
        c = torch.empty(M, N, device="cuda", dtype=bf)
        t = timeit(lambda: C.hgemm(a, w, c, M, N, K, K, K, N, True, True, cfg=0, splits=1))
        tf = 2.0 * M * N * K / t / 1e6
        print(json.dumps({"N": N, "tiles": tiles, "us": round(t, 1), "rounds": (tiles + 255) // 256,
                          "us_per_round": round(t / ((tiles + 255) // 256), 1), "TF": round(tf, 1)}), flush=True)
        del a, c
