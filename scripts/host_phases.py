#!/usr/bin/env python3
"""Host-side time of each phase of a training step (forward call, backward call, optimizer step, grad reset),
no syncs inside the step, against the GPU time of the whole step: when the host's total approaches the GPU's,
the GPU idles between kernels.  usage: host_phases.py [gpt2|resnet50] [steps]"""
import os, statistics, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_pytorch_example_amd.parallel import dist as pdist, DDP
from distributed_pytorch_example_amd.models import get_model
from distributed_pytorch_example_amd.optim import build_optimizer
from distributed_pytorch_example_amd.ops import functional as Fx
from distributed_pytorch_example_amd.utils.env import ensure_single_process_env

name = sys.argv[1] if len(sys.argv) > 1 else "gpt2"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
ensure_single_process_env()
pdist.init_process_group("auto")
dev = torch.device("cuda", 0)
model = get_model(name).to(dev)
ddp = DDP(model)
if name == "gpt2":
    opt = build_optimizer("adamw", model.parameters(), lr=6e-4, weight_decay=0.1)
    t = torch.randint(0, 50257, (8, 1025), device=dev)
    x, y = t[:, :-1].contiguous(), t[:, 1:].contiguous()
    fwd = lambda: ddp(x, y)
else:
    opt = build_optimizer("sgd", model.parameters(), lr=0.1, weight_decay=5e-5)
    x = torch.randn(512, 3, 224, 224, device=dev)
    y = torch.randint(0, 1000, (512,), device=dev)
    fwd = lambda: Fx.cross_entropy(ddp(x), y, 1000)
ph = {"fwd": [], "bwd": [], "opt": [], "reset": [], "gpu_step": []}
for i in range(steps + 5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter(); loss = fwd()
    t1 = time.perf_counter(); loss.backward()
    t2 = time.perf_counter(); opt.step()
    t3 = time.perf_counter()
    for p in model.parameters():
        p.grad = None
    t4 = time.perf_counter()
    e1.record()
    if i >= 5:
        ph["fwd"].append(t1 - t0); ph["bwd"].append(t2 - t1); ph["opt"].append(t3 - t2); ph["reset"].append(t4 - t3)
        e1.synchronize()
        ph["gpu_step"].append(e0.elapsed_time(e1) / 1e3)
print(name, " ".join(f"{k} {statistics.median(v) * 1e3:.3f} ms" for k, v in ph.items()), flush=True)
