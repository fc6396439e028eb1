#!/usr/bin/env python3
"""128-output-channel ResNet-50 GEMM shapes (layer-2 3x3 conv as a dense GEMM, batch 512) on each persistent-GEMM
tile (set_hgemm_force: 0 256x256, 1 128x256, 2 256x128, 3 128x128, -1 planner) against the implicit-GEMM conv."""
import json, os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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


C = ext()
bf = torch.bfloat16
for (M, K, N, label) in [(401408, 1152, 128, "L2 3x3 fwd"), (401408, 512, 128, "L2 1x1 512->128"),
                         (1605632, 256, 128, "L2.0 conv1 256->128 @56")]:
    a = torch.randn(M, K, device="cuda").to(bf)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(bf)
    fl = 2 * M * K * N
    res = {"shape": label, "M": M, "K": K, "N": N}
    for cfg in (-1, 0, 2, 3):
        C.set_hgemm_force(cfg, -1)
        try:
            t = timeit(lambda: C.linear_fwd(a, w))
            res[f"cfg{cfg}"] = round(t, 1)
        except Exception as e:  # noqa: BLE001
            res[f"cfg{cfg}"] = str(e)[:40]
    C.set_hgemm_force(-1, -1)
    print(json.dumps(res), flush=True)
    del a, w
    torch.cuda.empty_cache()
