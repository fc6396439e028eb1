#!/usr/bin/env python3
"""K-split sweep of the GPT-2 weight-grad GEMMs (TN, 256x256 tile, fp32 accumulate epilogue): time
of the whole call (split kernel + slab finalize) per split count, against the planner's pick.
One JSON line per shape.  python scripts/sweep_wgrad_splits.py"""
import json
import sys

import torch

sys.path.insert(0, ".")
from distributed_pytorch_example_amd.ops._ext import ext  # noqa: E402

sys.path.insert(0, "scripts")
from bench_hgemm import SHAPES, operands, timeit  # noqa: E402

C = ext()
for name, M, N, K, layout, epi, act in SHAPES:
    if layout != "wgrad":
        continue
    A, B, lda, ldb, ak, bk, _ = operands(M, N, K, layout)
    out = torch.zeros(M, N, device="cuda")
    plan = C.hgemm_plan(M, N, K, ak, bk, True, 4)
    res = {}
    for s in (1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 16):
        if K // 64 < 4 * s:
            continue
        try:
            res[s] = round(timeit(lambda: C.hgemm(A, B, out, M, N, K, lda, ldb, N, ak, bk, 2, 0, None, None, None, None,
                                                  1.0, 0, s)), 2)
        except RuntimeError:
            pass
    pick = round(timeit(lambda: C.hgemm(A, B, out, M, N, K, lda, ldb, N, ak, bk, 2, 0, None, None, None, None, 1.0, -1, -1)), 2)
    best = min(res, key=res.get)
    print(json.dumps({"gemm": name, "plan": list(plan)[:4], "us_planner": pick, "best_splits": best, "us_best": res[best],
                      "tflops_best": round(2 * M * N * K / res[best] / 1e6, 1), "us_by_splits": res}), flush=True)
