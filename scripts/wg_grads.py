#!/usr/bin/env python3
"""ResNet-50 gradients with the 1x1 conv weight grads on the implicit GEMM vs the persistent hgemm
kernel (same inputs, same weights): per-parameter relative difference and the loss."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_pytorch_example_amd.models import get_model
from distributed_pytorch_example_amd.ops import functional as Fx, ext

C = ext()
torch.manual_seed(0)
bs = int(sys.argv[1]) if len(sys.argv) > 1 else 64
model = get_model("resnet50").cuda()
x = Fx.to_s2d_input(torch.randn(bs, 3, 224, 224, device="cuda"))
y = torch.randint(0, 1000, (bs,), device="cuda")
grads = []
for on in (False, True, True):
    C.set_wgrad_hgemm(on)
    for p in model.parameters():
        p.grad = None
    loss = Fx.cross_entropy(model(x), y, 1000)
    loss.backward()
    torch.cuda.synchronize()
    grads.append({n: p.grad.detach().float().clone() for n, p in model.named_parameters()})
    print(f"hgemm={on} loss {loss.item():.6f}")
worst = []
for n in grads[0]:
    a, b, c = grads[0][n], grads[1][n], grads[2][n]
    r = ((a - b).norm() / (a.norm() + 1e-20)).item()
    rd = ((b - c).norm() / (b.norm() + 1e-20)).item()
    worst.append((r, rd, n, tuple(a.shape)))
worst.sort(reverse=True)
for r, rd, n, s in worst[:12]:
    print(f"{r:.3e}  (hgemm run-to-run {rd:.1e})  {n} {s}")
assert worst[0][0] < 1e-3, "wgrad routes disagree"
