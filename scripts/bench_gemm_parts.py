#!/usr/bin/env python3
"""Two-launch decompositions of the GPT-2 GEMMs (bindings/gemm.cpp plan2): a main part over whole
tile columns / rows that fills complete rounds of slots with one tile, plus a tail over the rest
with its own (smaller) tile, against the single-launch plans.  Measured with two hgemm calls on
sub-tensors (flat views: the sub-GEMMs' pointers are exactly plan2's), one JSON line per arm:

    python scripts/bench_gemm_parts.py [--only qkv.fwd]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from distributed_pytorch_example_amd.ops._ext import ext  # noqa: E402

sys.path.insert(0, "scripts")
from bench_hgemm import SHAPES, operands, timeit  # noqa: E402

C = ext()
TILES = {0: (256, 256), 1: (128, 256), 2: (256, 128), 3: (128, 128)}
LAYOK = {(True, True): [0, 1, 2, 3], (True, False): [0, 1], (False, False): [0]}

ap = argparse.ArgumentParser()
ap.add_argument("--only", default=None)
args = ap.parse_args()
ncu = torch.cuda.get_device_properties(0).multi_processor_count
for name, M, N, K, layout, epi, act in SHAPES:
    if args.only and args.only != name:
        continue
    if layout == "wgrad" or name.startswith("lmhead"):
        continue  # K-split plans / already multi-round: the decomposition targets the short-K forwards / dgrads
    A, B, lda, ldb, ak, bk, _ = operands(M, N, K, layout)
    odt = torch.float32 if epi else torch.bfloat16
    out = torch.empty(M, N, device="cuda", dtype=odt)

    def one(cfg, sp=1, M_=M, N_=N, Av=A, Bv=B, Cv=out):
        C.hgemm(Av, Bv, Cv, M_, N_, K, lda, ldb, N, ak, bk, epi, 0, None, None, None, None, 1.0, cfg, sp)

    res = {"gemm": name, "single_planner": round(timeit(lambda: one(-1, -1)), 1)}
    for cfg in LAYOK[(ak, bk)]:
        res[f"single_cfg{cfg}"] = round(timeit(lambda: one(cfg, 1)), 1)
    flatC = out.view(-1)
    for mc in LAYOK[(ak, bk)]:
        bm, bn = TILES[mc]
        bpc = 2 if mc == 3 else 1
        slots = ncu * bpc
        tm, tn = -(-M // bm), -(-N // bn)
        for axis in (0, 1):
            lines, per = (tn, tm) if axis == 0 else (tm, tn)
            rounds = lines * per // slots
            if rounds < 1:
                continue
            keep = rounds * slots // per
            at = keep * (bn if axis == 0 else bm)
            rest = (N if axis == 0 else M) - at
            if keep < 1 or rest < 64:
                continue
            for tc in LAYOK[(ak, bk)]:
                if axis == 0:
                    Bt = B[at:] if bk else B.view(-1)[at:]
                    Ct = flatC[at:]

                    def two():
                        one(mc, 1, M, at)
                        one(tc, -1, M, rest, A, Bt, Ct)
                else:
                    At = A[at:] if ak else A.view(-1)[at:]
                    Ct = flatC[at * N:]

                    def two():
                        one(mc, 1, at, N)
                        one(tc, -1, rest, N, At, B, Ct)
                res[f"two_axis{axis}_main{mc}_at{at}_tail{tc}"] = round(timeit(two), 1)
    p2 = C.hgemm_plan2(M, N, K, ak, bk, True, 4 if epi else 2)
    res["plan2"] = [p2[0][0], p2[1], p2[2], p2[3][0], round(p2[4], 1)]
    print(json.dumps(res), flush=True)
