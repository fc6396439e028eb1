# bf16-vs-fp32 gradient agreement as a function of batch size (noise should shrink ~1/sqrt(rows))
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import copy, torch
from distributed_pytorch_example_amd.models import get_model
from distributed_pytorch_example_amd.ops import functional as Fx
def rel(a,b): return ((a.float().cpu()-b.float().cpu()).norm()/(b.float().cpu().norm()+1e-12)).item()
def cos(a,b): a=a.float().cpu().flatten(); b=b.float().cpu().flatten(); return (a@b/(a.norm()*b.norm()+1e-12)).item()
for bs, hw in ((8, 64), (32, 64), (64, 96)):
    torch.manual_seed(0)
    cpu = get_model("resnet_tiny", num_classes=16)
    gpu = copy.deepcopy(cpu).cuda()
    x = torch.randn(bs, 3, hw, hw); y = torch.randint(0, 16, (bs,))
    lc = Fx.cross_entropy(cpu(x), y); lc.backward()
    lg = Fx.cross_entropy(gpu(x.cuda()), y.cuda()); lg.backward()
    gc = dict(cpu.named_parameters()); gg = dict(gpu.named_parameters())
    worst = max(((rel(gg[n].grad, gc[n].grad), n) for n in gc))
    mincos = min(((cos(gg[n].grad, gc[n].grad), n) for n in gc))
    print(f"bs={bs} hw={hw} loss cpu {lc.item():.4f} gpu {lg.item():.4f} worst-rel {worst[0]:.3f} ({worst[1]}) min-cos {mincos[0]:.4f} ({mincos[1]})")
