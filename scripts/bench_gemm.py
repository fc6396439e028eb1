#!/usr/bin/env python3
"""GEMM microbench on the GPT-2-small training shapes (tokens M = 8192):
ours (auto dispatch: 256-tile LDS-DMA kernel where eligible), ours with the
256-tile kernel disabled (128-tile igemm), and torch/hipBLASLt bf16 matmul.
Random non-zero operands (DVFS: zero data reads fast).  TF/s = 2MNK / time."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from distributed_pytorch_example_amd.ops._ext import ext  # noqa: E402

dev = "cuda"
C = ext()
T = 8192
SHAPES = [  # (name, kind, M, N, K) in GEMM terms
    ("qkv.fwd", "fwd", T, 2304, 768), ("proj.fwd", "fwd", T, 768, 768), ("fc.fwd", "fwd", T, 3072, 768),
    ("mproj.fwd", "fwd", T, 768, 3072), ("lmhead.fwd", "fwd", T, 50304, 768),
    ("qkv.dgrad", "dgrad", T, 768, 2304), ("fc.dgrad", "dgrad", T, 768, 3072), ("mproj.dgrad", "dgrad", T, 3072, 768),
    ("lmhead.dgrad", "dgrad", T, 768, 50304),
    ("qkv.wgrad", "wgrad", 2304, 768, T), ("proj.wgrad", "wgrad", 768, 768, T), ("fc.wgrad", "wgrad", 3072, 768, T),
    ("mproj.wgrad", "wgrad", 768, 3072, T), ("lmhead.wgrad", "wgrad", 50304, 768, T),
]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    out = []
    for name, kind, M, N, K in SHAPES:
        g = torch.Generator(device=dev).manual_seed(0)
        if kind == "fwd":
            x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
            w = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
            ours = lambda: C.linear_fwd(x, w, None, 0, False)  # noqa: E731
            ref = lambda: x @ w.t()  # noqa: E731
        elif kind == "dgrad":  # dx[M,N] = dy[M,K] @ w[K,N]
            dy = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
            w = (torch.randn(K, N, device=dev, generator=g) * 0.05).to(torch.bfloat16)
            ours = lambda: C.linear_dgrad(dy, w)  # noqa: E731
            ref = lambda: dy @ w  # noqa: E731
        else:  # dw[M,N] += dy[K,M]^T @ x[K,N]
            dy = torch.randn(K, M, device=dev, generator=g).to(torch.bfloat16)
            x = torch.randn(K, N, device=dev, generator=g).to(torch.bfloat16)
            dw = torch.zeros(M, N, device=dev)
            ours = lambda: C.linear_wgrad(dy, x, dw, 1.0)  # noqa: E731
            ref = lambda: dy.t() @ x  # noqa: E731
        fl = 2.0 * M * N * K
        C.set_gemm_backend(1)
        C.set_gemm256_mode(0)
        t_nat = timeit(ours)
        C.set_gemm256_mode(1)
        t_ig = timeit(ours)
        C.set_gemm256_mode(0)
        C.set_gemm_backend(2)
        t_lib = timeit(ours)
        C.set_gemm_backend(0)
        t_auto = timeit(ours)
        t_ref = timeit(ref)
        row = {"gemm": name, "M": M, "N": N, "K": K, "dispatch_us": round(t_auto * 1e6, 1),
               "dispatch_TF": round(fl / t_auto / 1e12, 1), "native_TF": round(fl / t_nat / 1e12, 1),
               "igemm128_TF": round(fl / t_ig / 1e12, 1), "lib_arm_TF": round(fl / t_lib / 1e12, 1),
               "torch_TF": round(fl / t_ref / 1e12, 1)}
        out.append(row)
        print(json.dumps(row), flush=True)
    tot = sum(r["dispatch_us"] for r in out)
    print(json.dumps({"total_ours_us_per_layer_set": round(tot, 1)}))


if __name__ == "__main__":
    main()
