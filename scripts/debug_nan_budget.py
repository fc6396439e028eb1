import copy, os, sys
sys.path.insert(0, os.getcwd())
import torch
from distributed_pytorch_example_amd.models import get_model
from distributed_pytorch_example_amd.ops import ext, functional as Fx
C = ext()
dev = "cuda"
torch.manual_seed(13)
base = get_model("resnet50").to(dev)
x = torch.randn(16, 3, 224, 224, device=dev)
y = torch.randint(0, 1000, (16,), device=dev)
for reserve in (0, 16):
    m = copy.deepcopy(base)
    C.set_cu_reserve(reserve)
    C.set_comm_active(reserve > 0)
    loss = Fx.cross_entropy(m(x), y, 1000)
    loss.backward()
    C.set_comm_active(False)
    C.set_cu_reserve(0)
    torch.cuda.synchronize()
    names = [n for n, p in m.named_parameters()]
    bad = [n for n, p in m.named_parameters() if p.grad is None or not torch.isfinite(p.grad).all()]
    print("reserve", reserve, "loss", loss.item(), "nonfinite", len(bad), "of", len(names))
    good = [n for n in names if n not in bad]
    print("  finite:", good[-12:])
    print("  first bad (reverse order):", [n for n in reversed(names) if n in bad][:8])
