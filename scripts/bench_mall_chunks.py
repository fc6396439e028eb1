#!/usr/bin/env python3
"""Does re-reading a tensor while it is resident in the 256 MiB Infinity Cache pay?  A 1x1
conv backward at ResNet-50 layer-1/2 sizes (weight grad then data grad, both reading dy):
whole tensors vs M-chunks sized so each dy chunk is re-read from MALL."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import statistics

import torch

from distributed_pytorch_example_amd.ops import ext


def timeit(fn, reps=10):
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
    for (N, HW, cin, cout) in [(512, 56, 64, 256), (512, 28, 128, 512), (512, 14, 256, 1024)]:
        x = torch.randn(N, HW, HW, cin, device=dev).to(torch.bfloat16)          # a2 (conv3 input)
        dy = torch.randn(N, HW, HW, cout, device=dev).to(torch.bfloat16)        # dh3
        w = (torch.randn(cout, 1, 1, cin, device=dev) / cin ** 0.5).to(torch.bfloat16)
        dw = torch.zeros(cout, 1, 1, cin, device=dev)

        def whole():
            C.conv_wgrad(dy, x, dw, [1, 1], [0, 0], [1, 1], 1.0)
            C.conv_dgrad(dy, w, [N, HW, HW, cin], [1, 1], [0, 0], [1, 1], None)

        res = {"whole": timeit(whole)}
        for nch in (2, 4, 8, 16):
            b = N // nch
            xs, dys = [x[i * b:(i + 1) * b] for i in range(nch)], [dy[i * b:(i + 1) * b] for i in range(nch)]

            def chunked():
                for xc, dc in zip(xs, dys):
                    C.conv_wgrad(dc, xc, dw, [1, 1], [0, 0], [1, 1], 1.0)
                    C.conv_dgrad(dc, w, [b, HW, HW, cin], [1, 1], [0, 0], [1, 1], None)

            res[f"chunks{nch}"] = timeit(chunked)
        mb = dy.numel() * 2 / 2**20
        print(f"N={N} HW={HW} {cin}->{cout} dy={mb:.0f}MiB " + " ".join(f"{k}={v:.1f}us" for k, v in res.items()))


if __name__ == "__main__":
    main()
