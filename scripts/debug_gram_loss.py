"""ResNet-50 step-0 loss and per-block BN3 statistics: ours with the Gram path on / off vs the fp32 torch twin."""
import copy
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import distributed_pytorch_example_amd.models._resnet_fused as rf  # noqa: E402
from distributed_pytorch_example_amd.models import get_model  # noqa: E402
from distributed_pytorch_example_amd.ops import functional as Fx  # noqa: E402
from test_model_parity_gpu import _TResNet  # noqa: E402

dev = torch.device("cuda")
torch.backends.cuda.matmul.allow_tf32 = False
torch.backends.cudnn.allow_tf32 = False
torch.manual_seed(0)
base = get_model("resnet50").to(dev)
twin = _TResNet(base).to(dev)
g = torch.Generator(device=dev).manual_seed(1)
x = torch.randn(8, 3, 224, 224, device=dev, generator=g)
y = torch.randint(0, 1000, (8,), device=dev, generator=g)
lt = F.cross_entropy(twin(x), y).item()
rm_t = [b.c3.bn.running_mean.clone() for b in twin.blocks]
rv_t = [b.c3.bn.running_var.clone() for b in twin.blocks]
for on in (False, True):
    rf._GRAM = on
    m = copy.deepcopy(base)
    lo = Fx.cross_entropy(m(x), y, 1000).item()
    dm = [((b.c3.bn.running_mean - r).norm() / (r.norm() + 1e-12)).item() for b, r in zip(m.blocks, rm_t)]
    dv = [((b.c3.bn.running_var - r).norm() / (r.norm() + 1e-12)).item() for b, r in zip(m.blocks, rv_t)]
    print(f"gram={on}: loss {lo:.5f} vs fp32 {lt:.5f} ({(lo - lt) / lt:+.2e})", flush=True)
    print("   BN3 running_mean rel dev per block:", " ".join(f"{v:.1e}" for v in dm))
    print("   BN3 running_var  rel dev per block:", " ".join(f"{v:.1e}" for v in dv))
