#!/usr/bin/env python3
"""How a training step reacts to foreign workgroups holding CU slots during backward -- a stand-in
for RCCL channel blocks overlapping the gradient all-reduce at 8 ranks.

Per step: forward on the compute stream; then a side stream launches `hogs` workgroups (threads,
LDS bytes and ~VGPRs per lane of an RCCL channel block, profiles/rccl_footprint_r3.txt) that stay
resident until the compute stream, after backward, sets their stop flag -- exactly the window in
which the reducer has bucket all-reduces in flight.  With `reserve` > 0 the persistent kernels plan
around `reserve` slots during that window (the CU budget the reducer applies at world > 1,
csrc/comm/comm.cpp); `set_comm_active` brackets the backward as Reducer::launch / finalize do.

    python scripts/hog_probe.py --model resnet50 --modes 0:0 16:0 16:16 0:16     (hogs:reserve pairs)
prints one JSON line per mode (median / min ms per step over alternating rounds)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_pytorch_example_amd.models import get_model  # noqa: E402
from distributed_pytorch_example_amd.ops import ext, functional as Fx  # noqa: E402
from distributed_pytorch_example_amd.optim import build_optimizer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="resnet50", choices=["resnet50", "gpt2"])
ap.add_argument("--batch-size", type=int, default=None)
ap.add_argument("--threads", type=int, default=256)
ap.add_argument("--lds", type=int, default=20480)
ap.add_argument("--vgprs", type=int, default=64)
ap.add_argument("--steps", type=int, default=6, help="timed steps per mode per round")
ap.add_argument("--sleepy", type=int, default=0,
                help="0: VALU-saturating hogs (worst case), 1: resident but idle (s_sleep), "
                     "2: RCCL-like reduce-copy streaming (two reads + one write per element, little VALU)")
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--modes", nargs="+", default=["0:0", "16:0", "16:16", "0:16"])
args = ap.parse_args()

C = ext()
dev = torch.device("cuda")
torch.manual_seed(0)
if args.model == "resnet50":
    bs = args.batch_size or 512
    model = get_model("resnet50").to(dev)
    opt = build_optimizer("sgd", model.parameters(), lr=0.1, weight_decay=5e-5)
    x = Fx.to_s2d_input(torch.randn(bs, 3, 224, 224, device=dev))
    y = torch.randint(0, 1000, (bs,), device=dev)

    def fwd():
        return Fx.cross_entropy(model(x), y, 1000)
else:
    bs = args.batch_size or 8
    model = get_model("gpt2").to(dev)
    opt = build_optimizer("adamw", model.parameters(), lr=1e-4, weight_decay=0.1)
    x = torch.randint(0, 50257, (bs, 1024), device=dev)
    y = torch.randint(0, 50257, (bs, 1024), device=dev)

    def fwd():
        return model(x, y)

side = torch.cuda.Stream()
stop = torch.zeros(1, dtype=torch.int32, device=dev)
modes = [tuple(int(v) for v in m.split(":")) for m in args.modes]


def step(hogs, reserve):
    loss = fwd()
    if hogs:
        C.hog_stop(stop, 0)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            C.cu_hog(hogs, args.threads, args.lds, 200000.0, args.vgprs, stop, mode=args.sleepy)  # bounded: 200 ms
    C.set_cu_reserve(reserve)
    C.set_comm_active(reserve > 0)
    loss.backward()
    C.set_comm_active(False)
    if hogs:
        C.hog_stop(stop, 1)
    opt.step()
    for p in model.parameters():
        p.grad = None


for _ in range(4):
    step(0, 0)
torch.cuda.synchronize()
res = {m: [] for m in modes}
for _ in range(args.rounds):
    for m in modes:
        step(*m)  # untimed: settles the allocator for this mode
        torch.cuda.synchronize()
        for _ in range(args.steps):
            t0 = time.perf_counter()
            step(*m)
            torch.cuda.synchronize()
            res[m].append((time.perf_counter() - t0) * 1e3)
C.set_cu_reserve(0)
base = None
for m in modes:
    ts = sorted(res[m])
    med = ts[len(ts) // 2]
    base = med if base is None else base
    print(json.dumps({"model": args.model, "batch": bs, "hogs": m[0], "reserve": m[1], "threads": args.threads,
                      "lds": args.lds, "vgprs": args.vgprs, "sleepy": args.sleepy, "ms_step_median": round(med, 3),
                      "ms_step_min": round(ts[0], 3), "vs_first_mode": round(med / base, 4)}), flush=True)
