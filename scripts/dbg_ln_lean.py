#!/usr/bin/env python3
"""LayerNorm forward / backward, lean vs generic kernels across processes (DPE_LN_FWD_LEAN / DPE_LN_BWD_LEAN
are read once per process):
`python scripts/dbg_ln_lean.py save <file>` under each setting, then `compare <a> <b>` (bitwise)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

if sys.argv[1] == "compare":
    a, b = torch.load(sys.argv[2], weights_only=True), torch.load(sys.argv[3], weights_only=True)
    for k in a:
        print(k, torch.equal(a[k], b[k]), (a[k].float() - b[k].float()).abs().max().item())
    sys.exit(0 if all(torch.equal(a[k], b[k]) for k in a) else 1)
from distributed_pytorch_example_amd.ops import ext  # noqa: E402

C = ext()
g = torch.Generator(device="cuda").manual_seed(5)
out = {}
for D, rows in ((768, 4100), (1024, 333)):
    dy = torch.randn(rows, D, device="cuda", generator=g).bfloat16()
    x = torch.randn(rows, D, device="cuda", generator=g) * 2 + 0.5
    w = torch.rand(D, device="cuda", generator=g) + 0.5
    mean = x.mean(1)
    rstd = torch.rsqrt(x.var(1, unbiased=False) + 1e-5)
    res = torch.randn(rows, D, device="cuda", generator=g)
    wb, bb = torch.zeros(D, device="cuda"), torch.zeros(D, device="cuda")
    dx, dxb = C.layernorm_bwd_residual(dy, x, w, mean, rstd, wb, bb, res)
    out[f"dx{D}"], out[f"dxb{D}"], out[f"dw{D}"], out[f"db{D}"] = dx, dxb, wb, bb
    bias = torch.randn(D, device="cuda", generator=g)
    for xx, nm in ((x, "f32"), (x.bfloat16(), "bf16")):
        yo = C.layernorm_fwd(xx, w, bias)
        for i, t in enumerate(yo if isinstance(yo, (list, tuple)) else [yo]):
            out[f"fwd{D}_{nm}_{i}"] = t
torch.save({k: v.cpu() for k, v in out.items()}, sys.argv[2])
