#!/usr/bin/env python3
"""Per-shape A/B of the persistent GEMM's dynamic unit claiming (hgemm.hip, set_hgemm_dynamic) on
the GPT-2-small GEMMs of scripts/bench_hgemm.py, planner's pick, arms interleaved 3 times; one JSON
line per GEMM (us per call, best of the interleaved rounds).  --reserve R marks a collective in
flight with a CU budget of R slots (more rounds per GEMM)."""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from distributed_pytorch_example_amd.ops._ext import ext  # noqa: E402

sys.path.insert(0, "scripts")
from bench_hgemm import SHAPES, operands, timeit  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reserve", type=int, default=0)
args = ap.parse_args()
C = ext()
C.set_cu_reserve(args.reserve)
C.set_comm_active(args.reserve > 0)
tot = {True: 0.0, False: 0.0}
for name, M, N, K, layout, epi, act in SHAPES:
    A, B, lda, ldb, ak, bk, _ = operands(M, N, K, layout)
    out = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16 if epi == 0 else torch.float32)
    aux = torch.randn(M, N, device="cuda").bfloat16() if act == 3 else None
    act_ = act if act == 3 else 0

    def one():
        C.hgemm(A, B, out, M, N, K, lda, ldb, N, ak, bk, epi, act_, None, None, aux, None, 1.0, -1, -1)

    best = {True: 1e30, False: 1e30}
    for _ in range(3):
        for d in (True, False):
            C.set_hgemm_dynamic(d)
            best[d] = min(best[d], timeit(one))
    for d in best:
        tot[d] += best[d]
    plan = C.hgemm_plan(M, N, K, ak, bk, layout == "wgrad", 2 if epi == 0 else 4)
    print(json.dumps({"gemm": name, "plan": list(plan), "us_dynamic": round(best[True], 2),
                      "us_static": round(best[False], 2), "ratio": round(best[True] / best[False], 4),
                      "reserve": args.reserve}), flush=True)
print(json.dumps({"total_us_dynamic": round(tot[True], 1), "total_us_static": round(tot[False], 1),
                  "reserve": args.reserve}), flush=True)
C.set_hgemm_dynamic(True)
C.set_comm_active(False)
C.set_cu_reserve(0)
