#!/usr/bin/env python3
"""Stream-K conv GEMM check (hgemm.hip SKM): the implicit-im2col 3x3 convs with SK on vs off -- outputs and BN
partials against each other and a torch fp32 conv, run-to-run bitwise determinism, then timing at batch 512."""
import json, os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from distributed_pytorch_example_amd.ops import ext

C = ext()
bf = torch.bfloat16


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


torch.manual_seed(0)
for ci, h, B in [(256, 14, 128), (256, 14, 512), (512, 7, 512)]:
    x = torch.randn(B, h, h, ci, device="cuda").to(bf)
    w = (torch.randn(ci, 3, 3, ci, device="cuda") / (9 * ci) ** 0.5).to(bf)
    ref = F.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), padding=1).permute(0, 2, 3, 1)
    C.set_hgemm_sk(False)
    y0, s0 = C.conv_fwd(x, w, [1, 1], [1, 1], [1, 1], True, None)
    t0 = timeit(lambda: C.conv_fwd(x, w, [1, 1], [1, 1], [1, 1], True, None))
    C.set_hgemm_sk(True)
    y1, s1 = C.conv_fwd(x, w, [1, 1], [1, 1], [1, 1], True, None)
    y2, s2 = C.conv_fwd(x, w, [1, 1], [1, 1], [1, 1], True, None)
    t1 = timeit(lambda: C.conv_fwd(x, w, [1, 1], [1, 1], [1, 1], True, None))
    torch.cuda.synchronize()
    e0 = ((y0.float() - ref).abs().max() / ref.abs().max()).item()
    e1 = ((y1.float() - ref).abs().max() / ref.abs().max()).item()
    st0 = s0.sum(-1); st1 = s1.sum(-1)
    print(json.dumps({"C": ci, "H": h, "B": B, "err_off": e0, "err_sk": e1, "det": bool(torch.equal(y1, y2) and torch.equal(s1, s2)),
                      "y_diff_frac": (y0 != y1).float().mean().item(),
                      "stats_rel": ((st0 - st1).abs().max() / st0.abs().max()).item(),
                      "us_off": round(t0, 1), "us_sk": round(t1, 1)}), flush=True)
