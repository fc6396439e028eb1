"""Block-by-block comparison of a ResNet forward with and without the on-load forward BN apply."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_pytorch_example_amd.models import _resnet_fused as RF
from distributed_pytorch_example_amd.models.resnet import ResNet

dev = torch.device("cuda")
torch.manual_seed(3)
model = ResNet((2, 2, 2, 1), num_classes=10).to(dev)
x = torch.randn(8, 3, 64, 64, device=dev)
outs = {}
orig = RF.BottleneckFn.forward


def rec(tag):
    def f(ctx, xx, block, link_in, link_out, defer_out, *params):
        out = orig(ctx, xx, block, link_in, link_out, defer_out, *params)
        outs.setdefault(tag, []).append((xx, out, ctx.saved_tensors if hasattr(ctx, "saved_tensors") else None))
        return out
    return f


for tag, f in (("ref", False), ("ax", True)):
    RF._AX_FWD = f
    RF.BottleneckFn.forward = staticmethod(rec(tag))
    with torch.no_grad():
        pass
    y = model(x)
    torch.cuda.synchronize()
    outs[tag + "_y"] = y.detach().clone()
    outs[tag + "_blocks"] = [(a.detach().clone(), b.detach().clone()) for a, b, _ in outs[tag]]
RF.BottleneckFn.forward = orig
for i, ((xa, oa), (xb, ob)) in enumerate(zip(outs["ref_blocks"], outs["ax_blocks"])):
    print(i, "in equal", torch.equal(xa, xb), "out equal", torch.equal(oa, ob),
          "in maxdiff", (xa.float() - xb.float()).abs().max().item(), "out maxdiff", (oa.float() - ob.float()).abs().max().item())
print("logits maxdiff", (outs["ref_y"] - outs["ax_y"]).abs().max().item())
