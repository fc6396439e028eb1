#!/usr/bin/env python3
"""How a training step reacts to foreign workgroups holding CU slots during backward -- a stand-in
for RCCL channel blocks overlapping the gradient all-reduce at 8 ranks.

Per step: forward on the compute stream; then a side stream launches `hogs` workgroups (threads,
LDS bytes and ~VGPRs per lane of an RCCL channel block, profiles/world8_1gpu_r6.txt) that stay
resident until the compute stream, after backward, sets their stop flag -- exactly the window in
which the reducer has bucket all-reduces in flight.  With `reserve` > 0 the persistent kernels plan
around `reserve` slots during that window (the CU budget the reducer applies at world > 1,
csrc/comm/comm.cpp); `set_comm_active` brackets the backward as Reducer::launch / finalize do.

    python scripts/hog_probe.py --model resnet50 --modes 0:0 16:0 16:16 0:16     (hogs:reserve pairs)
prints one JSON line per mode (median / min ms per step over alternating rounds).

Production path (default, --ddp 1): the model runs under DDP at world 1 with the W = 8 bucket layout
(parallel/buckets.py xgmi_bucket_policy(8)), so the gradients are bucket views, the overwrite-mode
first writes and GPT-2's grouped whole-round weight-grad launches are live exactly as in bench.py;
the windowed hogs start when the reducer issues a bucket (its transport's on_launch, index order), and
each round of --steps steps is timed as one window with no synchronisation inside it."""
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
ap.add_argument("--windowed", type=float, default=0.0,
                help="> 0: hogs resident only in the bucket all-reduce windows the W = 8 bucket policy predicts "
                     "(parallel/buckets.py): one hog launch per bucket when its gradients are ready, alive for "
                     "alpha + 2 (7/8) bytes / (this many GB/s of bus bandwidth) -- a model of RCCL's channel "
                     "blocks at 8 ranks instead of the whole-backward worst case")
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--modes", nargs="+", default=["0:0", "16:0", "16:16", "0:16"])
ap.add_argument("--ddp", type=int, default=1, help="1: through DDP (production path); 0: the bare model (round-5 probe)")
args = ap.parse_args()

C = ext()
dev = torch.device("cuda")
torch.manual_seed(0)
if args.model == "resnet50":
    bs = args.batch_size or 512
    model = get_model("resnet50").to(dev)
    opt = build_optimizer("sgd", model.parameters(), lr=0.1, weight_decay=5e-5)
    x = torch.randn(bs, 3, 224, 224, device=dev)
    y = torch.randint(0, 1000, (bs,), device=dev)

    def fwd():
        return Fx.cross_entropy(net(x), y, 1000)
else:
    bs = args.batch_size or 8
    model = get_model("gpt2").to(dev)
    opt = build_optimizer("adamw", model.parameters(), lr=1e-4, weight_decay=0.1)
    x = torch.randint(0, 50257, (bs, 1024), device=dev)
    y = torch.randint(0, 50257, (bs, 1024), device=dev)

    def fwd():
        return net(x, y)

net = model
ddp = None
if args.ddp:
    from distributed_pytorch_example_amd.parallel import DDP
    from distributed_pytorch_example_amd.parallel.buckets import xgmi_bucket_policy

    # world 1: no collectives, but the W = 8 bucket layout and every gradient-as-bucket-view path
    f8, c8, l8 = xgmi_bucket_policy(8, 4 * sum(p.numel() for p in model.parameters()))
    ddp = DDP(model, bucket_cap_mb=c8, first_bucket_mb=f8, last_bucket_mb=l8 or 0, rebuild_buckets=False)
    net = ddp
side = torch.cuda.Stream()
stop = torch.zeros(1, dtype=torch.int32, device=dev)
modes = [tuple(int(v) for v in m.split(":")) for m in args.modes]

# windowed: the W = 8 buckets (same policy and ready order as DDP: reverse registration order)
params = [p for p in model.parameters() if p.requires_grad]
win = {"on": False, "hogs": 0, "pending": [], "left": [], "reserve": 0}
if args.windowed > 0:
    from distributed_pytorch_example_amd.parallel.buckets import assign_buckets, xgmi_bucket_policy

    sizes = [p.numel() * 4 for p in params]
    f_mb, cap_mb, last_mb = xgmi_bucket_policy(8, sum(sizes))
    buckets = assign_buckets(sizes, list(range(len(params)))[::-1], int(cap_mb * 2**20), int(f_mb * 2**20),
                             None, int(last_mb * 2**20) if last_mb else None)
    bucket_of = {id(params[i]): b for b, idx in enumerate(buckets) for i in idx}
    bucket_us = [15.0 + 2 * 7 / 8 * sum(sizes[i] for i in idx) / (args.windowed * 1e3) for idx in buckets]
    print(json.dumps({"windowed_gbps": args.windowed, "buckets_mb": [round(sum(sizes[i] for i in idx) / 2**20, 2) for idx in buckets],
                      "window_us": [round(t, 1) for t in bucket_us]}), flush=True)

    def on_grad(p):
        if not win["on"]:
            return
        b = bucket_of.get(id(p))
        if b is None:
            return
        win["left"][b] -= 1
        if win["left"][b] == 0:  # the bucket's all-reduce would start now: hogs for its modelled duration
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                C.cu_hog(win["hogs"], args.threads, args.lds, bucket_us[b], args.vgprs, stop, mode=args.sleepy)

    def launch_window(b):
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            C.cu_hog(win["hogs"], args.threads, args.lds, bucket_us[b], args.vgprs, stop, mode=args.sleepy)

    if ddp is not None:
        # the reducer issues bucket b (index order, as the RCCL reducer would start its all-reduce)
        assert [list(i) for i in ddp.bucket_indices] == [list(i) for i in buckets], "bucket layout differs from the W=8 policy"
        tr = ddp._transport
        orig = tr.on_launch

        def on_launch(b, _orig=orig):
            if win["on"]:
                launch_window(b)
            if win["reserve"] > 0:
                C.set_comm_active(True)  # as Reducer::launch: the budget from the first bucket issue on
            return _orig(b)

        tr.on_launch = on_launch
        ddp.reducer = C.Reducer.host(ddp.buckets, ddp.bucket_indices, len(ddp._params), 1, tr.on_launch, tr.on_finalize)
    else:
        for p in params:
            p.register_post_accumulate_grad_hook(on_grad)


def step(hogs, reserve):
    loss = fwd()
    if hogs and args.windowed > 0:
        C.hog_stop(stop, 0)
        win.update(on=True, hogs=hogs, left=[len(idx) for idx in buckets])
    elif hogs:
        C.hog_stop(stop, 0)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            C.cu_hog(hogs, args.threads, args.lds, 200000.0, args.vgprs, stop, mode=args.sleepy)  # bounded: 200 ms
    C.set_cu_reserve(reserve)
    win["reserve"] = reserve
    if ddp is None or args.windowed <= 0:
        C.set_comm_active(reserve > 0)  # whole backward (DDP windowed: from the first bucket issue)
    loss.backward()
    C.set_comm_active(False)
    win["on"] = False
    if hogs:
        C.hog_stop(stop, 1)
        torch.cuda.current_stream().wait_stream(side)
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
        if args.ddp:  # one window of --steps steps, no synchronisation inside (as bench.py times)
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step(*m)
            torch.cuda.synchronize()
            res[m].append((time.perf_counter() - t0) * 1e3 / args.steps)
            continue
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
    print(json.dumps({"model": args.model, "ddp": args.ddp, "batch": bs, "hogs": m[0], "reserve": m[1], "windowed": args.windowed, "threads": args.threads,
                      "lds": args.lds, "vgprs": args.vgprs, "sleepy": args.sleepy, "ms_step_median": round(med, 3),
                      "ms_step_min": round(ts[0], 3), "vs_first_mode": round(med / base, 4)}), flush=True)
