"""Model-level GPU tests: the hand-scheduled ResNet bottleneck against the
per-op autograd path, and GPU (bf16 kernels) against the CPU fp32 reference
implementation of the same module with identical weights."""
import copy

import pytest
import torch
import torch.nn as nn

from distributed_pytorch_example_amd.models import get_model
from distributed_pytorch_example_amd.ops import functional as Fx

pytestmark = pytest.mark.gpu
dev = "cuda"


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def cos(a, b):
    a, b = a.float().flatten(), b.float().flatten()
    return (a @ b / (a.norm() * b.norm() + 1e-12)).item()


def _grads(model):
    return {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}


def test_fused_bottleneck_matches_per_op(C):
    """One bottleneck block (shallow => well conditioned): hand-scheduled fused
    fwd/bwd vs the per-op autograd path must agree tightly."""
    from distributed_pytorch_example_amd.models.resnet import Bottleneck

    torch.manual_seed(0)
    for inpl, planes, stride, down in [(64, 64, 1, True), (256, 64, 1, False), (256, 128, 2, True)]:
        b1 = Bottleneck(inpl, planes, stride, down).to(dev)
        b2 = copy.deepcopy(b1)
        b2.fused = False
        x = torch.randn(16, 28, 28, inpl, device=dev).to(torch.bfloat16)
        x1, x2 = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
        g = torch.randn(16, 28 // stride, 28 // stride, planes * 4, device=dev).to(torch.bfloat16)
        y1, y2 = b1(x1), b2(x2)
        assert rel(y1, y2) < 1e-2
        y1.backward(g)
        y2.backward(g)
        assert rel(x1.grad, x2.grad) < 3e-2
        for (n, p1), (_, p2) in zip(b1.named_parameters(), b2.named_parameters()):
            assert rel(p1.grad, p2.grad) < 3e-2, n
        for (n, r1), (_, r2) in zip(b1.named_buffers(), b2.named_buffers()):
            assert rel(r1, r2) < 1e-2, n


def test_chained_blocks_bn3_fusion_matches_per_op(C):
    """Blocks chained as in ResNet.forward: each identity block's first data-grad
    epilogue masks and reduces the PREVIOUS block's BN3 backward (_BN3Link)."""
    from distributed_pytorch_example_amd.models import _resnet_fused as RF
    from distributed_pytorch_example_amd.models.resnet import Bottleneck

    assert RF._BN3_CHAIN
    torch.manual_seed(5)
    cfg = [(64, 64, 1, True), (256, 64, 1, False), (256, 64, 1, False), (256, 128, 2, True), (512, 128, 1, False)]
    s1 = nn.ModuleList([Bottleneck(*c) for c in cfg]).to(dev)
    s2 = copy.deepcopy(s1)
    for b in s2:
        b.fused = False
    x = torch.randn(8, 28, 28, 64, device=dev).to(torch.bfloat16)
    x1, x2 = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    h1, link = x1, None
    for b in s1:
        h1, link = b.forward_chained(h1, link)
    h2 = x2
    for b in s2:
        h2 = b(h2)
    assert rel(h1, h2) < 2e-2
    g = torch.randn_like(h1)
    h1.backward(g)
    h2.backward(g)
    assert rel(x1.grad, x2.grad) < 5e-2
    for (n, p1), (_, p2) in zip(s1.named_parameters(), s2.named_parameters()):
        assert rel(p1.grad, p2.grad) < 5e-2, n


def test_resnet50_step_with_odd_layer4_input(C):
    """at 112x112 the layer-4 downsample block's input is [N, 7, 7, 1024] (odd H/W), so
    that block cannot chain the previous block's BN3 backward; the previous block must then NOT take the
    Gram path (it has no standalone BN3 backward).  A whole step runs and its gradients are finite."""
    torch.manual_seed(2)
    m = get_model("resnet50").to(dev)
    x = torch.randn(32, 3, 112, 112, device=dev)
    y = torch.randint(0, 1000, (32,), device=dev)
    loss = Fx.cross_entropy(m(x), y, 1000)
    loss.backward()
    torch.cuda.synchronize()
    assert torch.isfinite(loss).item()
    for n, p in m.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all().item(), n


def test_resnet_gpu_vs_cpu_reference(C):
    torch.manual_seed(1)
    cpu = get_model("resnet_tiny", num_classes=10)
    gpu = copy.deepcopy(cpu).to(dev)
    x = torch.randn(8, 3, 32, 32)
    y = torch.randint(0, 10, (8,))
    lc = Fx.cross_entropy(cpu(x), y)
    lc.backward()
    lg = Fx.cross_entropy(gpu(x.to(dev)), y.to(dev))
    lg.backward()
    assert abs(lc.item() - lg.item()) < 5e-2 * abs(lc.item())
    # bf16 rounding noise is amplified by every BN backward of a random-init net: the CPU
    # bf16-emulation (tests/test_numerics_cpu.py) shows the same ~0.4 worst-case deviation
    # from fp32, so deep layers are compared by direction and the head tightly.
    gc = {n: p.grad for n, p in cpu.named_parameters()}
    for n, p in gpu.named_parameters():
        assert cos(p.grad.cpu(), gc[n]) > 0.8, n
    assert rel(dict(gpu.named_parameters())["fc.bias"].grad.cpu(), gc["fc.bias"]) < 2e-2


@pytest.mark.parametrize("dtype,tol", [("fp32", 1e-5), ("bf16", 0.1)])
def test_simplenet_gpu_vs_cpu(C, dtype, tol):
    torch.manual_seed(2)
    cpu = get_model("simplenet")
    gpu = copy.deepcopy(cpu).to(dev)
    gpu.compute_dtype = dtype
    cpu.eval(); gpu.eval()  # dropout off for a deterministic comparison
    x = torch.randn(64, 784)
    y = torch.randint(0, 10, (64,))
    lc = Fx.cross_entropy(cpu(x), y)
    lc.backward()
    lg = Fx.cross_entropy(gpu(x.to(dev)), y.to(dev))
    lg.backward()
    assert abs(lc.item() - lg.item()) < (1e-5 if dtype == "fp32" else 2e-2)
    gc = {n: p.grad for n, p in cpu.named_parameters()}
    for n, p in gpu.named_parameters():  # bf16: ~5% on layers.0.weight (CPU bf16 emulation agrees)
        assert rel(p.grad.cpu(), gc[n]) < tol, n


def test_fused_optimizers_match_torch(C):
    from distributed_pytorch_example_amd.optim import SGD, Adam, AdamW

    torch.manual_seed(3)
    for ours_cls, ref_cls, kw in [(Adam, torch.optim.Adam, dict(lr=1e-2, weight_decay=0.01)),
                                  (AdamW, torch.optim.AdamW, dict(lr=1e-2, weight_decay=0.1)),
                                  (SGD, torch.optim.SGD, dict(lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)),
                                  (SGD, torch.optim.SGD, dict(lr=0.1))]:
        # 16-B vector body + ragged tails (37000, 70001) and a 4-B-misaligned
        # gradient view (scalar path), like a bucket view after an odd-sized param
        p1 = [torch.randn(1000, 37, device=dev, requires_grad=True), torch.randn(70001, device=dev, requires_grad=True),
              torch.randn(5000, device=dev, requires_grad=True)]
        p2 = [p.detach().clone().requires_grad_(True) for p in p1]
        o1, o2 = ours_cls(p1, **kw), ref_cls(p2, **kw)
        flat = torch.zeros(5001, device=dev)
        for _ in range(3):
            for a, b in zip(p1, p2):
                g = torch.randn_like(a)
                if a.numel() == 5000:
                    flat[1:].copy_(g)
                    a.grad = flat[1:]
                else:
                    a.grad = g.clone()
                b.grad = g.clone()
            o1.step(); o2.step()
        for a, b in zip(p1, p2):
            assert rel(a.detach(), b.detach()) < 1e-5, ours_cls.__name__
        sd = o1.state_dict()
        assert set(sd["param_groups"][0].keys()) == set(o2.state_dict()["param_groups"][0].keys())


def test_bf16_shadow_refreshed_by_fused_step(C):
    from distributed_pytorch_example_amd.ops import _state
    from distributed_pytorch_example_amd.optim import SGD

    p = torch.randn(64, 32, device=dev, requires_grad=True)
    sh = _state.shadow(p)
    opt = SGD([p], lr=0.5)
    p.grad = torch.ones_like(p)
    opt.step()
    assert torch.equal(_state.shadow(p), p.detach().to(torch.bfloat16))
    assert _state.shadow(p).data_ptr() == sh.data_ptr()


def test_gpt2_tiny_gpu_vs_cpu(C):
    torch.manual_seed(4)
    cpu = get_model("gpt2-tiny")
    gpu = copy.deepcopy(cpu).to(dev)
    idx = torch.randint(0, 512, (2, 128))
    tgt = torch.randint(0, 512, (2, 128))
    lc = Fx.cross_entropy(cpu(idx), tgt)
    lc.backward()
    lg = Fx.cross_entropy(gpu(idx.to(dev)), tgt.to(dev))
    lg.backward()
    assert abs(lc.item() - lg.item()) < 2e-2 * abs(lc.item())
    gc = dict(cpu.named_parameters())
    for n, p in gpu.named_parameters():
        assert cos(p.grad.cpu(), gc[n].grad) > 0.98, n
        assert rel(p.grad.cpu(), gc[n].grad) < 0.1, n


def test_gpt2_fused_lm_head_ce(C):
    """model(idx, targets) (fused LM head + in-place CE + alpha-scaled GEMMs) == unfused logits + CE."""
    torch.manual_seed(7)
    m1 = get_model("gpt2-tiny").to(dev)
    m2 = copy.deepcopy(m1)
    idx = torch.randint(0, 512, (2, 128), device=dev)
    tgt = torch.randint(0, 512, (2, 128), device=dev)
    l1 = Fx.cross_entropy(m1(idx), tgt)
    (3.0 * l1).backward()
    l2 = m2(idx, tgt)
    (3.0 * l2).backward()
    assert abs(l1.item() - l2.item()) < 1e-3 * abs(l1.item())
    g1 = dict(m1.named_parameters())
    for n, p in m2.named_parameters():
        assert cos(p.grad, g1[n].grad) > 0.999, n
        assert rel(p.grad, g1[n].grad) < 0.02, n


def test_gpt2_small_step(C):
    from distributed_pytorch_example_amd.optim import AdamW

    torch.manual_seed(5)
    m = get_model("gpt2").to(dev)
    assert sum(p.numel() for p in m.parameters()) == 124439808
    opt = AdamW(m.parameters(), lr=3e-4, weight_decay=0.1)
    idx = torch.randint(0, 50257, (2, 1024), device=dev)
    losses = []
    for _ in range(3):
        loss = m(idx, idx)  # fused LM head + CE; learn the identity: loss must drop
        loss.backward()
        opt.step()
        for p in m.parameters():
            p.grad = None
        losses.append(loss.item())
    # ~ln(50257)=10.8 minus the tied-embedding self-similarity bonus of predicting the input token
    assert 9.0 < losses[0] < 11.5 and losses[-1] < losses[0]


def test_gpt2_fused_block_matches_per_op(C):
    """Hand-scheduled transformer block (one autograd node, residual-form LN backward with
    the bf16 gradient copy carried between blocks) == per-op autograd graph."""
    torch.manual_seed(8)
    for bias in (True, False):
        m1 = get_model("gpt2-tiny", n_layer=3, bias=bias).to(dev)
        m2 = copy.deepcopy(m1)
        for b in m2.h:
            b.fused = False
        assert all(b.fused for b in m1.h)
        idx = torch.randint(0, 512, (2, 128), device=dev)
        tgt = torch.randint(0, 512, (2, 128), device=dev)
        l1, l2 = m1(idx, tgt), m2(idx, tgt)
        assert abs(l1.item() - l2.item()) < 1e-4 * abs(l2.item())
        l1.backward()
        l2.backward()
        g2 = dict(m2.named_parameters())
        for n, p in m1.named_parameters():
            assert cos(p.grad, g2[n].grad) > 0.999, n
            assert rel(p.grad, g2[n].grad) < 0.02, n


def test_resnet_counts_batches_once_per_forward(C):
    """The fused ResNet advances every BatchNorm's num_batches_tracked once per training forward
    (one multi-tensor launch for all blocks; a standalone block still counts its own)."""
    from distributed_pytorch_example_amd.models import get_model

    torch.manual_seed(3)
    model = get_model("resnet18_like").to(dev)
    x = torch.randn(4, 3, 32, 32, device=dev)
    for _ in range(2):
        model(x)
    counts = {n: int(b.item()) for n, b in model.named_buffers() if n.endswith("num_batches_tracked")}
    assert counts and all(v == 2 for v in counts.values()), counts


@pytest.mark.parametrize("reserve", [0, 16])
def test_resnet_bn_statistics_bitwise_reproducible(C, reserve):
    """BatchNorm statistics come from per-tile / per-row-group partials in fixed layouts and are summed
    in a fixed order, so two identical training forwards give bitwise-equal running statistics and
    BN-backward sums -- also while the CU budget is active (reserve > 0: the persistent kernels run
    with fewer row groups, a different but equally fixed partial layout)."""
    from distributed_pytorch_example_amd.models import get_model
    from distributed_pytorch_example_amd.ops import functional as Fx

    torch.manual_seed(13)
    base = get_model("resnet50").to(dev)
    x = torch.randn(16, 3, 224, 224, device=dev)
    y = torch.randint(0, 1000, (16,), device=dev)
    outs = []
    C.set_cu_reserve(reserve)
    try:
        for _ in range(2):
            m = copy.deepcopy(base)
            C.set_comm_active(reserve > 0)
            loss = Fx.cross_entropy(m(x), y, 1000)
            loss.backward()
            C.set_comm_active(False)
            torch.cuda.synchronize()
            stats = [b.detach().clone() for n, b in m.named_buffers() if "running" in n]
            bn_grads = [(n, p.grad.detach().clone()) for n, p in m.named_parameters() if ".bn." in n]
            outs.append((loss.item(), stats, bn_grads))
    finally:
        C.set_comm_active(False)
        C.set_cu_reserve(0)
    (l1, s1, g1), (l2, s2, g2) = outs
    assert l1 == l2
    assert len(s1) == 2 * 53 and all(torch.equal(a, b) for a, b in zip(s1, s2))
    bad = [(n, (a - b).abs().max().item()) for (n, a), (_, b) in zip(g1, g2) if not torch.equal(a, b)]
    assert not bad, bad


def test_graph_replayed_step_matches_eager(C):
    """A whole SimpleNet training step (forward, fused CE, backward, fused Adam with its device-side
    step counters and hyper-parameters) captured once in a HIP graph and replayed == the same steps
    run eagerly (the bench.py --graph path, without the DDP wrapper)."""
    from distributed_pytorch_example_amd.models import get_model
    from distributed_pytorch_example_amd.ops import functional as Fx
    from distributed_pytorch_example_amd.optim import Adam

    torch.manual_seed(11)
    m1 = get_model("simplenet").to(dev)
    m1.layers[2].p = m1.layers[5].p = 0.0  # dropout seeds come from a host counter: a replay reuses its masks
    m2 = copy.deepcopy(m1)
    o1, o2 = Adam(m1.parameters(), lr=1e-3), Adam(m2.parameters(), lr=1e-3)
    xs = [torch.randn(64, 784, device=dev) for _ in range(5)]
    ys = [torch.randint(0, 10, (64,), device=dev) for _ in range(5)]

    def step(model, opt, x, y):
        loss = Fx.cross_entropy(model(x), y, 10)
        loss.backward()
        opt.step()
        # gradients stay allocated (zeroed in place): the fused optimizer's device table holds their
        # pointers, which a graph replay must find unchanged (under DDP they are the bucket views)
        opt.zero_grad(set_to_none=False)
        return loss

    for m in (m1, m2):
        for p in m.parameters():
            p.grad = torch.zeros_like(p)
    step(m1, o1, xs[0], ys[0])  # eager warm-up step on both (optimizer state exists before capture)
    step(m2, o2, xs[0], ys[0])
    sx, sy = xs[1].clone(), ys[1].clone()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        step(m1, o1, sx, sy)  # step 2 on the side stream (capture warm-up)
    torch.cuda.current_stream().wait_stream(side)
    o1.graph_safe = True
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        gl = step(m1, o1, sx, sy)  # captured (this does not run step 3)
    step(m2, o2, xs[1], ys[1])
    for i in (2, 3, 4):
        sx.copy_(xs[i])
        sy.copy_(ys[i])
        g.replay()
        l2 = step(m2, o2, xs[i], ys[i])
    torch.cuda.synchronize()
    assert abs(gl.item() - l2.item()) <= 1e-4 * max(1.0, abs(l2.item()))
    for (n, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        assert rel(a.detach(), b.detach()) < 1e-4, n
