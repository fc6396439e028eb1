#!/usr/bin/env python3
"""How the ResNet-50 step reacts to foreign workgroups holding CU slots (a stand-in for RCCL
channel blocks overlapping the backward at 8 ranks).  Each step, a side stream launches
`nblocks` hog workgroups (threads / LDS per block configurable) that stay resident for the whole
step; the compute stream runs forward + backward + SGD.  Prints ms/step per configuration."""
import os, sys, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_pytorch_example_amd.models import get_model
from distributed_pytorch_example_amd.ops import functional as Fx, ext
from distributed_pytorch_example_amd.optim import build_optimizer

C = ext()
dev = torch.device("cuda")
torch.manual_seed(0)
bs = 512
model = get_model("resnet50").to(dev)
opt = build_optimizer("sgd", model.parameters(), lr=0.1, weight_decay=5e-5)
x = Fx.to_s2d_input(torch.randn(bs, 3, 224, 224, device=dev))
y = torch.randint(0, 1000, (bs,), device=dev)
side = torch.cuda.Stream()
confs = [tuple(int(v) for v in c.split(":")) for c in (sys.argv[1:] or ["0:256:0", "16:256:0", "32:256:0", "64:256:0"])]


def step():
    loss = Fx.cross_entropy(model(x), y, 1000)
    loss.backward()
    opt.step()
    for p in model.parameters():
        p.grad = None


for _ in range(6):
    step()
torch.cuda.synchronize()
for rep in range(2):
    for nb, th, lds in confs:
        ts = []
        for i in range(8):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if nb:
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    C.cu_hog(nb, th, lds, 60000.0 if i < 7 else 45000.0)
            step()
            torch.cuda.current_stream().synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
            torch.cuda.synchronize()  # hog drains before the next step
        ts.sort()
        print(json.dumps({"hog_blocks": nb, "threads": th, "lds": lds, "ms_step_median": round(ts[len(ts) // 2], 3),
                          "ms_step_min": round(ts[0], 3)}), flush=True)
