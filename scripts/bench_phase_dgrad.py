#!/usr/bin/env python3
"""Strided 3x3 data grads (4 per-parity sub-GEMMs, with and without the BN-backward epilogue) under each
LDS-DMA conv tile (set_conv_tile: 0 auto, 1 128-row, 2 256x128, 3 256x256), batch 512.  CUDA-event
timing, min over alternating rounds of median-of-20."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_pytorch_example_amd.ops import ext  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


C = ext()
B = int(os.environ.get("B", "512"))
modes = [int(m) for m in os.environ.get("MODES", "0,2,3").split(",")]
for (ci, co, h) in [(128, 128, 56), (256, 256, 28), (512, 512, 14)]:
    ho = h // 2
    w = (torch.randn(co, 3, 3, ci, device="cuda") / (9 * ci) ** 0.5).to(torch.bfloat16)
    dy = torch.randn(B, ho, ho, co, device="cuda").to(torch.bfloat16)
    hh = torch.randn(B, h, h, ci, device="cuda").to(torch.bfloat16)
    coef = torch.stack([torch.rand(ci, device="cuda") + 0.5, torch.randn(ci, device="cuda") * 0.1,
                        torch.randn(ci, device="cuda") * 0.1, torch.rand(ci, device="cuda") + 0.5]).contiguous()
    xs = [B, h, h, ci]
    ref = None
    res = {}
    for _ in range(3):
        for m in modes:
            C.set_conv_tile(m)
            for bnb in (False, True):
                if bnb:
                    f = lambda: C.conv_dgrad_bn(dy, w, xs, [2, 2], [1, 1], [1, 1], None, hh, coef)
                else:
                    f = lambda: C.conv_dgrad(dy, w, xs, [2, 2], [1, 1], [1, 1], None)
                res.setdefault((m, bnb), []).append(timeit(f))
            out = C.conv_dgrad_bn(dy, w, xs, [2, 2], [1, 1], [1, 1], None, hh, coef)
            dx, part = out[0].float(), out[1].sum(-1)
            if ref is None:
                ref = (dx, part)
            else:  # same values whatever the tile (partials summed over tiles)
                assert torch.allclose(dx, ref[0], atol=1e-2, rtol=1e-2), f"mode {m}: dx differs"
                assert torch.allclose(part, ref[1], atol=1e-1, rtol=1e-2), f"mode {m}: partials differ"
    C.set_conv_tile(0)
    print(f"{ci}->{co} 3x3/s2 @{h}: " + "  ".join(f"tile{m}{'+bnb' if b else ''} {min(v):.1f}" for (m, b), v in res.items()),
          flush=True)
