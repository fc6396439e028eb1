#!/usr/bin/env python3
"""On-load BN apply (conv1x1_bnin_fwd / _dgrad) vs the standalone pass + conv it replaces, at the
ResNet-50 batch-512 shapes of layers 1-4.  CUDA-event timing, median of reps; prints JSON lines."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributed_pytorch_example_amd.ops import ext


def timeit(fn, reps=10):
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


def coef(c):
    return torch.stack([torch.rand(c, device="cuda") + 0.5, torch.randn(c, device="cuda") * 0.5,
                        torch.randn(c, device="cuda") * 0.3, torch.rand(c, device="cuda") + 0.5]).contiguous()


def main():
    C = ext()
    B = int(os.environ.get("BATCH", "512"))
    bf = torch.bfloat16
    for H, Cin, Cm in [(56, 256, 64), (28, 512, 128), (14, 1024, 256), (7, 2048, 512)]:
        h = torch.randn(B, H, H, Cin, device="cuda").to(bf)
        res = torch.randn(B, H, H, Cin, device="cuda").to(bf)
        c3, cd = coef(Cin), coef(Cin)
        w1 = (torch.randn(Cm, 1, 1, Cin, device="cuda") / Cin ** 0.5).to(bf)
        x = torch.empty_like(h)
        bits = torch.empty(B, H, H, Cin // 8, dtype=torch.uint8, device="cuda")
        for down in (False, True):
            rc = cd if down else None
            t_ref = timeit(lambda: C.conv_fwd(C.bn_apply(h, c3, res, rc, True, True)[0], w1, [1, 1], [0, 0], [1, 1], True, None))
            t_app = timeit(lambda: C.bn_apply(h, c3, res, rc, True, True))
            for tile in ((128, 256) if Cm == 64 else (128,)):
                t_ax = timeit(lambda: C.conv1x1_bnin_fwd(h, res, c3, rc, w1, x, bits, True, tile))
                print(json.dumps({"op": "fwd", "H": H, "Cin": Cin, "Cout": Cm, "down": down, "tile": tile,
                                  "ref_us": round(t_ref, 1), "apply_us": round(t_app, 1), "ax_us": round(t_ax, 1)}), flush=True)
        # backward: conv3 (Cm -> Cin) data grad over dh3 = a dz3 + b h3 + c
        dz = res
        w3 = (torch.randn(Cin, 1, 1, Cm, device="cuda") / Cin ** 0.5).to(bf)
        h2 = torch.randn(B, H, H, Cm, device="cuda").to(bf)
        c2 = coef(Cm)
        gamma = torch.rand(Cin, device="cuda") + 0.5
        part = torch.randn(2, Cin, 64, device="cuda")
        bco = C.bn_bwd_coef(part, h.numel() // Cin, gamma, c3, None, None)
        dh = torch.empty_like(h)

        def ref():
            d = C.bn_bwd_partials(dz, h, gamma, c3, part, None, None, relu_mask=False)
            C.conv_dgrad_bn(d, w3, [B, H, H, Cm], [1, 1], [0, 0], [1, 1], None, h2, c2)

        t_ref = timeit(ref)
        t_app = timeit(lambda: C.bn_bwd_partials(dz, h, gamma, c3, part, None, None, relu_mask=False))
        t_ax = timeit(lambda: C.conv1x1_bnin_dgrad(dz, h, bco, w3, dh, h2, c2))
        print(json.dumps({"op": "dgrad", "H": H, "Cin": Cin, "Cout": Cm, "ref_us": round(t_ref, 1),
                          "apply_us": round(t_app, 1), "ax_us": round(t_ax, 1)}), flush=True)
        del h, res, x, bits, dz, dh, h2
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
