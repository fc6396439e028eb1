#!/usr/bin/env python3
"""Achieved HBM bandwidth of the BatchNorm elementwise kernels at ResNet-50 batch-512 shapes
(bn_apply: read x, write y; bn_bwd_partials: read dz, x, write dx).  Random data, CUDA events."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import statistics

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


def main():
    C = ext()
    dev = "cuda"
    print(f"{'M':>9s} {'C':>5s} {'pass':14s} {'us':>8s} {'TB/s':>6s}")
    for M, Ch in [(512 * 56 * 56, 64), (512 * 56 * 56, 256), (512 * 28 * 28, 128), (512 * 28 * 28, 512),
                  (512 * 14 * 14, 256), (512 * 14 * 14, 1024), (512 * 7 * 7, 512), (512 * 7 * 7, 2048)]:
        x = torch.randn(M, Ch, device=dev).to(torch.bfloat16)
        r = torch.randn(M, Ch, device=dev).to(torch.bfloat16)
        coef = torch.stack([torch.rand(Ch, device=dev) + 0.5, torch.randn(Ch, device=dev),
                            torch.randn(Ch, device=dev), torch.rand(Ch, device=dev) + 0.5]).contiguous()
        nbytes = M * Ch * 2
        us = timeit(lambda: C.bn_apply(x, coef, None, None, True, False))
        print(f"{M:9d} {Ch:5d} {'apply':14s} {us:8.1f} {2 * nbytes / us / 1e6:6.2f}")
        us = timeit(lambda: C.bn_apply(x, coef, r, None, True, True))
        print(f"{M:9d} {Ch:5d} {'apply+res+bits':14s} {us:8.1f} {(3 * nbytes + nbytes / 16) / us / 1e6:6.2f}")
        part = torch.randn(2, Ch, 4, device=dev)
        g = torch.rand(Ch, device=dev)
        dg, db = torch.zeros(Ch, device=dev), torch.zeros(Ch, device=dev)
        us = timeit(lambda: C.bn_bwd_partials(r, x, g, coef, part, dg, db))
        print(f"{M:9d} {Ch:5d} {'bwd_apply':14s} {us:8.1f} {3 * nbytes / us / 1e6:6.2f}")
        us = timeit(lambda: r.copy_(x))
        print(f"{M:9d} {Ch:5d} {'torch copy':14s} {us:8.1f} {2 * nbytes / us / 1e6:6.2f}")


if __name__ == "__main__":
    main()
