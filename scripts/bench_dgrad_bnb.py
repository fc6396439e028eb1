#!/usr/bin/env python3
"""Layer-2 3x3 data grad with and without the BN-backward epilogue (EPI_BF16_BNB: reads the pre-BN
input h for the ReLU mask and the (sum dz, sum dz (h - mean)) partials) vs the forward conv of the same
shape, batch 512.  CUDA-event timing, median of N reps, alternating."""
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
for (ci, co, h, st) in [(128, 128, 28, 1), (256, 256, 14, 1), (64, 64, 56, 1), (128, 128, 56, 2), (256, 256, 28, 2),
                        (512, 512, 14, 2)]:
    if len(sys.argv) > 1 and sys.argv[1] == "strided" and st == 1:
        continue
    ho = h // st
    x = torch.randn(B, h, h, ci, device="cuda").to(torch.bfloat16)
    w = (torch.randn(co, 3, 3, ci, device="cuda") / (9 * ci) ** 0.5).to(torch.bfloat16)
    dy = torch.randn(B, ho, ho, co, device="cuda").to(torch.bfloat16)
    hh = torch.randn(B, h, h, ci, device="cuda").to(torch.bfloat16)
    coef = torch.stack([torch.rand(ci, device="cuda") + 0.5, torch.randn(ci, device="cuda") * 0.1,
                        torch.randn(ci, device="cuda") * 0.1, torch.rand(ci, device="cuda") + 0.5]).contiguous()
    arms = {
        "fwd+stats": lambda: C.conv_fwd(x, w, [st, st], [1, 1], [1, 1], True, None),
        "dgrad": lambda: C.conv_dgrad(dy, w, list(x.shape), [st, st], [1, 1], [1, 1], None),
        "dgrad+bnb": lambda: C.conv_dgrad_bn(dy, w, list(x.shape), [st, st], [1, 1], [1, 1], None, hh, coef),
    }
    res = {k: [] for k in arms}
    for _ in range(3):
        for k, f in arms.items():
            res[k].append(timeit(f))
    print(f"{ci}->{co} 3x3/s{st} @{h}: " + "  ".join(f"{k} {min(v):.1f} us" for k, v in res.items()), flush=True)
