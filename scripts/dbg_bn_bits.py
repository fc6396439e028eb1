import os, sys, torch
sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from distributed_pytorch_example_amd.ops import ext
C = ext()
dev = "cuda"
def bf(t): return t.to(torch.bfloat16)
torch.manual_seed(17)
N, H, W, Ci = 4, 14, 14, 256
h = bf(torch.randn(N, H, W, Ci, device=dev))
mean = h.float().mean((0, 1, 2)); var = h.float().var((0, 1, 2), unbiased=False)
inv = torch.rsqrt(var + 1e-5); g0 = torch.rand(Ci, device=dev) + 0.5; b0 = torch.randn(Ci, device=dev) * 0.1
coef = torch.stack([g0 * inv, b0 - mean * g0 * inv, mean, inv]).contiguous()
res = bf(torch.randn(N, H, W, Ci, device=dev))
y, bits = C.bn_apply(h, coef, res, None, True, True)
dy = bf(torch.randn(N, H, W, Ci, device=dev))
gamma = torch.rand(Ci, device=dev) + 0.5
outs = []
for use_bits in (False, True):
    dg, db = torch.zeros(Ci, device=dev), torch.zeros(Ci, device=dev)
    dx, dz = C.bn_bwd(dy, y, h, gamma, coef, dg, db, True, bits if use_bits else None)
    outs.append((dx, dz, dg, db))
for name, a, b in zip(["dx", "dz", "dg", "db"], *outs):
    print(os.environ.get("DPE_EXT_SO", "new"), name, torch.equal(a, b), (a.float() - b.float()).abs().max().item(), (a.float() != b.float()).sum().item())
