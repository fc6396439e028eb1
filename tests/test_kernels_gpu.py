"""Numerics of every gfx950 kernel against a plain fp32 PyTorch reference of the
same op (inputs rounded to bf16 first, so only accumulation/output rounding
differs).  Random NON-zero data throughout."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"


def bf(x):
    return x.to(torch.bfloat16)


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def test_extension_is_native(C):
    assert C.ARCH == "gfx950"


# ------------------------------------------------------------------ GEMMs
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (256, 192, 96), (1000, 520, 784), (64, 64, 32), (300, 1000, 2048),
                                   (8, 24, 40)])
def test_linear_fwd(C, M, N, K):
    torch.manual_seed(0)
    x = bf(torch.randn(M, K, device=dev))
    w = bf(torch.randn(N, K, device=dev) / math.sqrt(K))
    b = torch.randn(N, device=dev)
    ref = x.float() @ w.float().t() + b
    y = C.linear_fwd(x, w, b, 0, False)
    assert y.dtype == torch.bfloat16 and rel_err(y, ref) < 1e-2
    y32 = C.linear_fwd(x, w, b, 1, True)
    assert rel_err(y32, F.relu(ref)) < 1e-3


def test_linear_fwd_asymmetric_layout(C):
    # integer data: exact; catches row/col swaps in the C write
    M, N, K = 64, 64, 64
    x = torch.zeros(M, K, device=dev)
    x[torch.arange(M), torch.arange(M) % K] = 1.0
    w = (torch.arange(N * K, device=dev).reshape(N, K) % 7).float()
    y = C.linear_fwd(bf(x), bf(w), None, 0, True)
    assert torch.equal(y, (x @ w.t()))


@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (256, 192, 96), (1000, 784, 520), (64, 256, 16 * 8)])
def test_linear_dgrad(C, M, N, K):
    torch.manual_seed(1)
    dy = bf(torch.randn(M, N, device=dev))
    w = bf(torch.randn(N, K, device=dev))
    ref = dy.float() @ w.float()
    assert rel_err(C.linear_dgrad(dy, w), ref) < 1e-2


@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (4096, 256, 128), (100, 64, 64), (2048, 1000 // 8 * 8, 2048)])
def test_linear_wgrad(C, M, N, K):
    torch.manual_seed(2)
    dy = bf(torch.randn(M, N, device=dev))
    x = bf(torch.randn(M, K, device=dev))
    dw = torch.zeros(N, K, device=dev)
    C.linear_wgrad(dy, x, dw, 1.0)
    ref = dy.float().t() @ x.float()
    assert rel_err(dw, ref) < 1e-3
    C.linear_wgrad(dy, x, dw, 0.5)  # accumulate
    assert rel_err(dw, 1.5 * ref) < 1e-3


@pytest.mark.parametrize("M,N,K", [(1024, 3072, 768), (2048, 768, 3072), (512, 256, 192)])
def test_linear_wgrad_split_k(C, M, N, K):
    """Weight grads over a long token axis: K-split fp32 slabs + accumulate into the bucket."""
    torch.manual_seed(3)
    dy = bf(torch.randn(M, N, device=dev))
    x = bf(torch.randn(M, K, device=dev))
    dw = torch.randn(N, K, device=dev)
    ref = dw + dy.float().t() @ x.float()
    C.linear_wgrad(dy, x, dw, 1.0)
    torch.cuda.synchronize()
    assert rel_err(dw, ref) < 1e-3
    C.linear_wgrad(dy, x, dw, 0.5)
    assert rel_err(dw, ref + 0.5 * (dy.float().t() @ x.float())) < 1e-3


@pytest.mark.parametrize("M", [64, 50])
@pytest.mark.parametrize("act", [0, 1])
def test_linear_padded_out_features_fwd_bwd(C, M, act):
    """A Linear whose out_features is not a multiple of 8 (SimpleNet's 10-class head): bias + ReLU in
    the GEMM epilogue on the padded shadow, weight grad and fused bias grad written only for the N
    real rows from a column-padded dy (hgemm at M % 64 == 0, the implicit GEMM otherwise)."""
    from distributed_pytorch_example_amd.ops import functional as Fx

    torch.manual_seed(9)
    N, K = 10, 256
    lin = torch.nn.Linear(K, N).to(dev)
    w = lin.weight.detach().clone().requires_grad_(True)
    b = lin.bias.detach().clone().requires_grad_(True)
    x = bf(torch.randn(M, K, device=dev)).requires_grad_(True)
    y = Fx.linear(x, w, b, act, True)
    ref_w, ref_b = bf(w.detach()).float().requires_grad_(True), b.detach().clone().requires_grad_(True)
    xr = x.detach().float().requires_grad_(True)
    ref = F.linear(xr, ref_w, ref_b)
    ref = F.relu(ref) if act else ref
    assert y.shape == (M, N) and rel_err(y, ref) < 1e-2
    g = torch.randn(M, N, device=dev)
    y.backward(g)
    ref.backward(bf(g).float())
    assert rel_err(w.grad, ref_w.grad) < 1e-2 and rel_err(b.grad, ref_b.grad) < 1e-2
    assert rel_err(x.grad, xr.grad) < 1e-2


def test_linear_gelu_fused_fwd_bwd(C):
    """fc: u = gelu(x w^T + b) with the pre-activation v from the same epilogue; the next layer's
    data grad times gelu'(v) in its epilogue (GPT-2 MLP)."""
    torch.manual_seed(9)
    M, K, H = 1024, 256, 1024
    x = bf(torch.randn(M, K, device=dev))
    w = bf(torch.randn(H, K, device=dev) / math.sqrt(K))
    b = torch.randn(H, device=dev) * 0.1
    v = torch.empty(M, H, device=dev, dtype=torch.bfloat16)
    u = C.linear_fwd(x, w, b, 2, False, None, None, v)
    pre = x.float() @ w.float().t() + b
    assert rel_err(v, pre) < 1e-2
    assert rel_err(u, F.gelu(pre, approximate="tanh")) < 1e-2
    w2 = bf(torch.randn(K, H, device=dev) / math.sqrt(H))
    dy = bf(torch.randn(M, K, device=dev))
    dv = C.linear_dgrad(dy, w2, None, None, v)
    vv = v.float().requires_grad_(True)
    gg = torch.autograd.grad(F.gelu(vv, approximate="tanh").sum(), vv)[0]
    assert rel_err(dv, (dy.float() @ w2.float()) * gg) < 1e-2


# ------------------------------------------------------------------- conv
CONV_CASES = [
    # N, H, W, Cin, Cout, k, stride, pad
    (2, 8, 8, 64, 64, 1, 1, 0),
    (2, 8, 8, 64, 64, 3, 1, 1),
    (2, 14, 14, 128, 128, 3, 2, 1),
    (2, 14, 14, 256, 512, 1, 2, 0),
    (2, 28, 28, 8, 64, 7, 2, 3),     # stem (channel-padded input)
    (3, 7, 7, 512, 128, 3, 1, 1),
    (1, 9, 9, 32, 48, 3, 2, 1),
    (2, 10, 10, 16, 32, 5, 1, 2),    # stride-1 data grad as a forward conv (pad R-1-p)
    (2, 9, 9, 64, 64, 3, 1, 0),
    # ResNet-50 shapes at small batch (LDS-DMA kernel: M / N tails, 3-stage ring, strided 1x1)
    (2, 56, 56, 64, 256, 1, 1, 0),
    (2, 28, 28, 128, 128, 3, 1, 1),
    (2, 56, 56, 256, 512, 1, 2, 0),
    (5, 7, 7, 512, 512, 3, 1, 1),
    (3, 14, 14, 96, 200, 3, 1, 1),
    # write-heavy pointwise convs on the streaming kernel (pwconv.hip): K 64 / 128 / 256, M tails
    (1, 5, 5, 64, 256, 1, 1, 0),
    (3, 7, 7, 128, 512, 1, 1, 0),
    (2, 9, 9, 256, 1024, 1, 1, 0),
    (4, 30, 30, 64, 512, 1, 1, 0),
    # 1x1 data grad with K = 2048, M tail (588 rows)
    (3, 14, 14, 512, 2048, 1, 1, 0),
    # 1x1 forwards at depth >= 1024 (persistent GEMM with the BN-forward statistics epilogue), M tails
    (2, 7, 7, 1024, 256, 1, 1, 0),
    (3, 9, 9, 2048, 512, 1, 1, 0),
    # C = 16 (s2d stem form): two filter taps per 32-wide K-step on the LDS-DMA kernel
    (2, 12, 12, 16, 64, 4, 1, 2),
    (2, 9, 9, 16, 48, 2, 2, 0),
]


def _conv_ref(x, w, s, p):
    return F.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), None, s, p).permute(0, 2, 3, 1)


@pytest.mark.parametrize("N,H,W,Ci,Co,k,s,p", CONV_CASES)
def test_conv_fwd(C, N, H, W, Ci, Co, k, s, p):
    torch.manual_seed(3)
    x = bf(torch.randn(N, H, W, Ci, device=dev))
    w = bf(torch.randn(Co, k, k, Ci, device=dev) / math.sqrt(k * k * Ci))
    ref = _conv_ref(x, w, s, p)
    y, stats = C.conv_fwd(x, w, [s, s], [p, p], [1, 1], True, None)
    assert y.shape == ref.shape and rel_err(y, ref) < 1e-2
    yf = y.float().reshape(-1, Co)
    tot = stats.sum(-1)
    assert rel_err(tot[0], yf.sum(0)) < 1e-3
    assert rel_err(tot[1], (yf * yf).sum(0)) < 1e-3


@pytest.mark.parametrize("N,H,W,Ci,Co,k,s,p", [c for c in CONV_CASES if c[3] != 8])
def test_conv_dgrad(C, N, H, W, Ci, Co, k, s, p):
    torch.manual_seed(4)
    x = torch.randn(N, Ci, H, W, device=dev, requires_grad=True)
    w = bf(torch.randn(Co, k, k, Ci, device=dev) / math.sqrt(k * k * Ci))
    y = F.conv2d(x, w.permute(0, 3, 1, 2).float(), None, s, p)
    dy = bf(torch.randn_like(y))
    (ref,) = torch.autograd.grad(y, x, dy.float())
    dx = C.conv_dgrad(dy.permute(0, 2, 3, 1).contiguous(), w, [N, H, W, Ci], [s, s], [p, p], [1, 1], None)
    assert rel_err(dx, ref.permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.parametrize("N,H,W,Ci,Co,k,s,p", CONV_CASES)
def test_conv_wgrad(C, N, H, W, Ci, Co, k, s, p):
    torch.manual_seed(5)
    x = bf(torch.randn(N, H, W, Ci, device=dev))
    w = torch.randn(Co, Ci, k, k, device=dev, requires_grad=True)
    y = F.conv2d(x.permute(0, 3, 1, 2).float(), w, None, s, p)
    dy = bf(torch.randn_like(y))
    (ref,) = torch.autograd.grad(y, w, dy.float())
    dw = torch.zeros(Co, k, k, Ci, device=dev)
    C.conv_wgrad(dy.permute(0, 2, 3, 1).contiguous(), x, dw, [s, s], [p, p], [1, 1], 1.0)
    assert rel_err(dw, ref.permute(0, 2, 3, 1)) < 1e-3


@pytest.mark.parametrize("N,H,Ci,Co", [(4, 8, 128, 256), (16, 14, 256, 1024), (64, 28, 512, 128), (64, 7, 512, 2048),
                                       (8, 28, 128, 512)])
def test_conv_wgrad_pointwise_hgemm(C, N, H, Ci, Co):
    # 1x1 weight grads with pixels % 64 == 0 and both channel counts >= 128 run on the persistent
    # hgemm kernel (TN, K split over the pixels + slab finalize); accumulate with alpha
    torch.manual_seed(15)
    x = bf(torch.randn(N, H, H, Ci, device=dev))
    dy = bf(torch.randn(N, H, H, Co, device=dev))
    ref = dy.float().reshape(-1, Co).t() @ x.float().reshape(-1, Ci)
    init = torch.randn(Co, 1, 1, Ci, device=dev)
    dw = init.clone()
    C.conv_wgrad(dy, x, dw, [1, 1], [0, 0], [1, 1], 0.5)
    assert rel_err(dw.reshape(Co, Ci), init.reshape(Co, Ci) + 0.5 * ref) < 1e-3
    dw.zero_()
    C.conv_wgrad(dy, x, dw, [1, 1], [0, 0], [1, 1], 1.0)
    assert rel_err(dw.reshape(Co, Ci), ref) < 1e-3


def test_resnet_scale_shapes(C):
    # a real ResNet-50 layer1 shape at batch 32: fwd/dgrad/wgrad
    torch.manual_seed(6)
    N, H, Ci, Co = 32, 56, 64, 256
    x = bf(torch.randn(N, H, H, Ci, device=dev))
    w = bf(torch.randn(Co, 1, 1, Ci, device=dev) / 8)
    y, _ = C.conv_fwd(x, w, [1, 1], [0, 0], [1, 1], False, None)
    assert rel_err(y, _conv_ref(x, w, 1, 0)) < 1e-2
    dy = bf(torch.randn_like(y.float()))
    dw = torch.zeros(Co, 1, 1, Ci, device=dev)
    C.conv_wgrad(dy, x, dw, [1, 1], [0, 0], [1, 1], 1.0)
    ref = dy.float().reshape(-1, Co).t() @ x.float().reshape(-1, Ci)
    assert rel_err(dw.reshape(Co, Ci), ref) < 1e-3


# -------------------------------------------------------------- BatchNorm
@pytest.mark.parametrize("M,Cc,relu,res", [(4096, 64, True, False), (1000, 256, False, True), (98, 2048, True, True),
                                          (50000, 128, True, False)])
def test_bn_train_fwd_bwd(C, M, Cc, relu, res):
    torch.manual_seed(7)
    x = bf(torch.randn(M, Cc, device=dev) * 2 + 0.5)
    g = torch.rand(Cc, device=dev) + 0.5
    b = torch.randn(Cc, device=dev)
    r = bf(torch.randn(M, Cc, device=dev)) if res else None
    rm, rv = torch.zeros(Cc, device=dev), torch.ones(Cc, device=dev)
    y, coef = C.bn_fwd_train(x, g, b, rm, rv, 0.1, 1e-5, relu, r, None)
    xf = x.float().requires_grad_(True)
    gf, bfp = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    rf = r.float().requires_grad_(True) if res else None
    rm2, rv2 = torch.zeros(Cc, device=dev), torch.ones(Cc, device=dev)
    ref = F.batch_norm(xf, rm2, rv2, gf, bfp, True, 0.1, 1e-5)
    if res:
        ref = ref + rf
    if relu:
        ref = F.relu(ref)
    assert rel_err(y, ref) < 1e-2
    assert rel_err(rm, rm2) < 1e-4 and rel_err(rv, rv2) < 1e-4
    dy = bf(torch.randn(M, Cc, device=dev))
    grads = torch.autograd.grad(ref, [xf, gf, bfp] + ([rf] if res else []), dy.float())
    dg, db = torch.zeros(Cc, device=dev), torch.zeros(Cc, device=dev)
    dx, dz = C.bn_bwd(dy, y if relu else None, x, g, coef, dg, db, res)
    assert rel_err(dx, grads[0]) < 2e-2
    assert rel_err(dg, grads[1]) < 1e-2 and rel_err(db, grads[2]) < 1e-2
    if res:
        assert rel_err(dz, grads[3]) < 1e-2


def test_bn_stats_from_conv_epilogue(C):
    torch.manual_seed(8)
    x = bf(torch.randn(4, 16, 16, 64, device=dev))
    w = bf(torch.randn(128, 3, 3, 64, device=dev) / 24)
    y, st = C.conv_fwd(x, w, [1, 1], [1, 1], [1, 1], True, None)
    g, b = torch.ones(128, device=dev), torch.zeros(128, device=dev)
    y1, c1 = C.bn_fwd_train(y, g, b, None, None, 0.1, 1e-5, True, None, None)
    y2, c2 = C.bn_fwd_train(y, g, b, None, None, 0.1, 1e-5, True, None, st)
    assert rel_err(c1, c2) < 1e-4 and rel_err(y1, y2) < 1e-2


def test_bn_eval(C):
    x = bf(torch.randn(500, 64, device=dev))
    g, b = torch.rand(64, device=dev), torch.randn(64, device=dev)
    rm, rv = torch.randn(64, device=dev), torch.rand(64, device=dev) + 0.5
    y = C.bn_fwd_eval(x, g, b, rm, rv, 1e-5, True, None)
    ref = F.relu(F.batch_norm(x.float(), rm, rv, g, b, False, 0.1, 1e-5))
    assert rel_err(y, ref) < 1e-2


# ---------------------------------------------------------------- pooling
def test_maxpool(C):
    torch.manual_seed(9)
    x = bf(torch.randn(2, 17, 17, 64, device=dev))
    y, idx = C.maxpool_fwd(x, 3, 2, 1)
    xf = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    ref = F.max_pool2d(xf, 3, 2, 1)
    assert torch.equal(y.float(), ref.permute(0, 2, 3, 1))
    dy = bf(torch.randn_like(y.float()))
    (g,) = torch.autograd.grad(ref, xf, dy.float().permute(0, 3, 1, 2))
    dx = C.maxpool_bwd(dy, idx, list(x.shape), 3, 2, 1)
    assert rel_err(dx, g.permute(0, 2, 3, 1)) < 1e-2


def test_gavgpool(C):
    x = bf(torch.randn(4, 7, 7, 2048, device=dev))
    y = C.gavgpool_fwd(x)
    assert rel_err(y, x.float().mean((1, 2))) < 1e-2
    dy = bf(torch.randn(4, 2048, device=dev))
    dx = C.gavgpool_bwd(dy, list(x.shape))
    assert rel_err(dx, (dy.float() / 49)[:, None, None, :].expand(4, 7, 7, 2048)) < 1e-2


# ------------------------------------------------------------------- loss
@pytest.mark.parametrize("B,V,ld,in_bf", [(64, 16, 16, False), (256, 1000, 1000, False), (32, 50257, 50304, True),
                                         (16, 3000, 3000, True), (8, 100000, 100000, True)])
def test_cross_entropy(C, B, V, ld, in_bf):
    torch.manual_seed(10)
    z = torch.randn(B, ld, device=dev) * 3
    if in_bf:
        z = bf(z)
    y = torch.randint(0, V, (B,), device=dev)
    zf = z.float()[:, :V].requires_grad_(True)
    ref = F.cross_entropy(zf, y, reduction="sum")
    (g,) = torch.autograd.grad(ref, zf)
    rows, s, correct, d = C.cross_entropy(z, y, V, 1.0, True, in_bf, -100)
    assert abs(s.item() - ref.item()) / abs(ref.item()) < 1e-4
    assert correct.item() == (zf.argmax(1) == y).sum().item()
    assert rel_err(d[:, :V], g) < 1e-2
    if ld > V:
        assert d[:, V:].float().abs().max().item() == 0
    # in-place (row held in registers): gradient overwrites the logits
    z2 = z.clone()
    _, s2, _, d2 = C.cross_entropy(z2, y, V, 1.0, True, in_bf, -100, True)
    assert d2.data_ptr() == z2.data_ptr() and abs(s2.item() - s.item()) <= 1e-5 * abs(s.item())
    assert torch.equal(d2, d)


def test_cross_entropy_loss_sum_bitwise_reproducible(C):
    """The loss sum is a fixed-order reduction of the per-row losses (no float atomics): identical
    inputs give identical bits on every call, and it equals the rows' sum in that order's tolerance."""
    torch.manual_seed(11)
    z = bf(torch.randn(4096, 1000, device=dev) * 3)
    y = torch.randint(0, 1000, (4096,), device=dev)
    sums = [C.cross_entropy(z, y, 1000, 1.0, False, True, -100)[1].item() for _ in range(8)]
    assert len(set(sums)) == 1, sums
    rows = C.cross_entropy(z, y, 1000, 1.0, False, True, -100)[0]
    assert abs(rows.double().sum().item() - sums[0]) <= 1e-5 * abs(sums[0])


# ---------------------------------------------------------------- eltwise
def test_cast_act_dropout(C):
    x = torch.randn(1000003, device=dev)
    assert torch.equal(C.cast_bf16(x, None), x.to(torch.bfloat16))
    xb = bf(torch.randn(4096, 64, device=dev))
    assert torch.equal(C.act(xb, None, 0), F.relu(xb))
    g = C.act(xb, None, 2)
    assert rel_err(g, F.gelu(xb.float(), approximate="tanh")) < 1e-2
    dy = bf(torch.randn_like(xb.float()))
    xr = xb.float().requires_grad_(True)
    (ref,) = torch.autograd.grad(F.gelu(xr, approximate="tanh"), xr, dy.float())
    assert rel_err(C.act(dy, xb, 3), ref) < 2e-2
    y = C.dropout(torch.ones(100000, device=dev), 0.2, 1234, 0)
    keep = (y != 0).float().mean().item()
    assert abs(keep - 0.8) < 0.01 and torch.allclose(y[y != 0], torch.full_like(y[y != 0], 1.25))
    y2 = C.dropout(torch.ones(100000, device=dev), 0.2, 1234, 0)
    assert torch.equal(y, y2)


@pytest.mark.parametrize("M,N,dt", [(3000, 520, torch.bfloat16), (8192, 768, torch.float32), (8192, 3072, torch.bfloat16),
                                    (100, 36, torch.float32), (7, 1000, torch.bfloat16)])
def test_colsum(C, M, N, dt):
    dy = torch.randn(M, N, device=dev).to(dt)
    db = torch.full((N,), 7.0, device=dev)
    C.colsum(dy, db, False)  # overwrite
    assert rel_err(db, dy.float().sum(0)) < 1e-4
    C.colsum(dy, db, True)  # accumulate
    assert rel_err(db, 2 * dy.float().sum(0)) < 1e-4


@pytest.mark.parametrize("D", [768, 64, 1024, 2048, 4096, 5120, 6400])
def test_layernorm(C, D):
    torch.manual_seed(11)
    x = torch.randn(333, D, device=dev) * 2 + 1
    w, b = torch.rand(D, device=dev) + 0.5, torch.randn(D, device=dev)
    y, mean, rstd = C.layernorm_fwd(x, w, b, 1e-5)
    xf = x.clone().requires_grad_(True)
    wf, bfp = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    ref = F.layer_norm(xf, (D,), wf, bfp, 1e-5)
    assert rel_err(y, ref) < 1e-2
    # backward: D > 2048 runs full-row sums + <= 2048-column slices (norm.hip)
    dy = bf(torch.randn(333, D, device=dev))
    gx, gw, gb = torch.autograd.grad(ref, [xf, wf, bfp], dy.float())
    dw, db = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
    dx = C.layernorm_bwd(dy, x, w, mean, rstd, dw, db, None)
    assert rel_err(dx, gx) < 1e-2 and rel_err(dw, gw) < 1e-3 and rel_err(db, gb) < 1e-3
    acc = torch.ones(333, D, device=dev)
    C.layernorm_bwd(dy, x, w, mean, rstd, torch.zeros(D, device=dev), None, acc)
    assert rel_err(acc - 1, gx) < 1e-2


def test_layernorm_bwd_deferred_grouped_finalize(C):
    """The residual-stream LayerNorm backward with its dw / db reduction deferred (partials returned) and
    several LayerNorms' partials reduced by one grouped launch (GPT-2 two per block, norm.hip
    ln_bwd_finalize_group_kernel): bitwise the per-LayerNorm finalize, dx untouched by the deferral;
    mixed widths, one problem without a bias, accumulation into non-zero gradients."""
    torch.manual_seed(17)
    probs = []
    for rows, D, with_b in ((333, 768, True), (256, 64, False), (97, 1024, True), (512, 768, True)):
        x = torch.randn(rows, D, device=dev) * 2 + 1
        w, b = torch.rand(D, device=dev) + 0.5, torch.randn(D, device=dev)
        _, mean, rstd = C.layernorm_fwd(x, w, b, 1e-5)
        dy = bf(torch.randn(rows, D, device=dev))
        res = torch.randn(rows, D, device=dev)
        probs.append((x, w, mean, rstd, dy, res, with_b))
    ref, parts, outs = [], [], []
    for x, w, mean, rstd, dy, res, with_b in probs:
        D = x.shape[-1]
        dw, db = torch.full((D,), 0.5, device=dev), (torch.full((D,), -0.25, device=dev) if with_b else None)
        dx, dxb = C.layernorm_bwd_residual(dy, x, w, mean, rstd, dw, db, res)
        ref.append((dx, dxb, dw, db))
        dw2, db2 = torch.full((D,), 0.5, device=dev), (torch.full((D,), -0.25, device=dev) if with_b else None)
        dx2, dxb2, part = C.layernorm_bwd_residual(dy, x, w, mean, rstd, dw2, db2, res, True)
        assert torch.equal(dw2, torch.full((D,), 0.5, device=dev))  # untouched until the finalize
        parts.append(part)
        outs.append((dx2, dxb2, dw2, db2))
    C.layernorm_bwd_finalize_group(parts, [p[0].shape[0] for p in probs], [o[2] for o in outs], [o[3] for o in outs])
    for (dx, dxb, dw, db), (dx2, dxb2, dw2, db2) in zip(ref, outs):
        assert torch.equal(dx, dx2) and torch.equal(dxb, dxb2) and torch.equal(dw, dw2)
        assert (db is None and db2 is None) or torch.equal(db, db2)


def test_embedding(C):
    idx = torch.randint(0, 1000, (4, 64), device=dev)
    wte, wpe = bf(torch.randn(1000, 128, device=dev)), bf(torch.randn(64, 128, device=dev))
    out = C.embedding_fwd(idx, wte, wpe)
    assert rel_err(out, wte.float()[idx] + wpe.float()[None]) < 1e-6
    dout = torch.randn(4, 64, 128, device=dev)
    dwte, dwpe = torch.zeros(1000, 128, device=dev), torch.zeros(64, 128, device=dev)
    C.embedding_bwd(idx, dout, dwte, dwpe)
    ref = torch.zeros(1000, 128, device=dev).index_add_(0, idx.reshape(-1), dout.reshape(-1, 128))
    assert rel_err(dwte, ref) < 1e-5 and rel_err(dwpe, dout.sum(0)) < 1e-5


# -------------------------------------------------------------- attention
@pytest.mark.parametrize("B,T,H", [(2, 128, 2), (1, 1024, 3), (2, 256, 12)])
def test_attention_fwd_bwd(C, B, T, H):
    torch.manual_seed(12)
    D = 64
    qkv = bf(torch.randn(B, T, 3, H, D, device=dev))
    scale = 1.0 / math.sqrt(D)
    out, lse = C.attn_fwd(qkv, H, scale, True)
    q, k, v = qkv.float().permute(2, 0, 3, 1, 4).requires_grad_(True).unbind(0)
    qf, kf, vf = [t.detach().clone().requires_grad_(True) for t in (q, k, v)]
    ref = F.scaled_dot_product_attention(qf, kf, vf, is_causal=True)  # [B,H,T,D]
    assert rel_err(out.permute(0, 2, 1, 3), ref) < 1e-2
    # lse2 = log2-domain logsumexp of the scaled scores
    s = (qf @ kf.transpose(-1, -2)) * scale
    s = s.masked_fill(torch.triu(torch.ones(T, T, device=dev, dtype=torch.bool), 1), float("-inf"))
    assert rel_err(lse, torch.logsumexp(s, -1) / math.log(2)) < 1e-4
    do = bf(torch.randn(B, T, H, D, device=dev))
    gq, gk, gv = torch.autograd.grad(ref, [qf, kf, vf], do.float().permute(0, 2, 1, 3))
    dqkv = C.attn_bwd(qkv, out, do, lse, H, scale, True)
    for i, g in enumerate((gq, gk, gv)):
        assert rel_err(dqkv[:, :, i].permute(0, 2, 1, 3), g) < 2e-2, i


# ----------------------------- Linear GEMMs on the persistent MFMA kernel (hgemm.hip)
def test_linear_plain_paths(C):
    """The only GEMM backend is native: set_gemm_backend(1) is accepted, the library arm is gone."""
    C.set_gemm_backend(1)
    with pytest.raises(RuntimeError):
        C.set_gemm_backend(2)
    torch.manual_seed(8)
    M, N, K = 1024, 776, 512
    x = bf(torch.randn(M, K, device=dev))
    w = bf(torch.randn(N, K, device=dev) / math.sqrt(K))
    b = torch.randn(N, device=dev)
    assert rel_err(C.linear_fwd(x, w, b, 0, False), x.float() @ w.float().t() + b) < 1e-2
    dy = bf(torch.randn(M, N, device=dev))
    s = torch.tensor([0.5], device=dev)
    assert rel_err(C.linear_dgrad(dy, w, None, s), 0.5 * (dy.float() @ w.float())) < 1e-2
    dw = torch.randn(N, K, device=dev)
    ref = dw + 0.5 * (dy.float().t() @ x.float())
    C.linear_wgrad(dy, x, dw, 1.0, s)
    assert rel_err(dw, ref) < 1e-3
    # fp32 residual stream: y = res + x @ w^T + b
    res = torch.randn(M, N, device=dev)
    y = C.linear_fwd(x, w, b, 0, True, res)
    assert rel_err(y, res + x.float() @ w.float().t() + b) < 1e-4
    # column-padded dy (vocab-padded LM head): only the first N columns are real
    dyp = bf(torch.randn(M, N + 56, device=dev))
    dw2 = torch.zeros(N, K, device=dev)
    C.linear_wgrad(dyp, x, dw2, 1.0)
    assert rel_err(dw2, dyp[:, :N].float().t() @ x.float()) < 1e-3
    # odd vocabulary (N % 8 != 0) over a padded dy, as the tied LM head
    Nv = 771
    dyv = bf(torch.randn(M, 776, device=dev))
    dyv[:, Nv:] = 0
    dw3 = torch.zeros(Nv, K, device=dev)
    C.linear_wgrad(dyv, x, dw3, 1.0)
    assert rel_err(dw3, dyv[:, :Nv].float().t() @ x.float()) < 1e-3


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 256), (8192 // 8 + 64, 2304 // 4 + 8, 768), (300, 520, 128)])
def test_linear_fwd_epilogues(C, M, N, K):
    torch.manual_seed(3)
    x = bf(torch.randn(M, K, device=dev))
    w = bf(torch.randn(N, K, device=dev) / math.sqrt(K))
    b = torch.randn(N, device=dev)
    ref = x.float() @ w.float().t() + b
    y = C.linear_fwd(x, w, b, 0, False)
    assert rel_err(y, ref) < 1e-2
    yg = C.linear_fwd(x, w, b, 2, False)  # fused tanh-GELU epilogue
    assert rel_err(yg, F.gelu(ref, approximate="tanh")) < 1e-2
    res = torch.randn(M, N, device=dev)
    y32 = C.linear_fwd(x, w, b, 0, True, res)  # fp32 out + fp32 residual
    assert rel_err(y32, ref + res) < 1e-4
    rb = bf(torch.randn(M, N, device=dev))
    yr = C.linear_fwd(x, w, None, 0, False, rb)  # bf16 residual
    assert rel_err(yr, x.float() @ w.float().t() + rb.float()) < 1e-2


def test_linear_asymmetric_layout_persistent(C):
    M, N, K = 256, 256, 128
    x = torch.zeros(M, K, device=dev)
    x[torch.arange(M), torch.arange(M) % K] = 1.0
    w = (torch.arange(N * K, device=dev).reshape(N, K) % 7).float()
    assert torch.equal(C.linear_fwd(bf(x), bf(w), None, 0, True), x @ w.t())
    # dgrad layout (B N-contiguous): dx = dy @ w
    dy = (torch.arange(M * N, device=dev).reshape(M, N) % 5).float()
    w2 = torch.zeros(N, K, device=dev)
    w2[torch.arange(N), torch.arange(N) % K] = 1.0
    assert torch.equal(C.linear_dgrad(bf(dy), bf(w2)).float(), dy @ w2)


@pytest.mark.parametrize("M,N,K", [(512, 256, 768), (1024, 768, 2304), (320, 520, 192)])
def test_linear_dgrad_persistent(C, M, N, K):
    torch.manual_seed(4)
    dy = bf(torch.randn(M, N, device=dev))
    w = bf(torch.randn(N, K, device=dev))
    assert rel_err(C.linear_dgrad(dy, w), dy.float() @ w.float()) < 1e-2


@pytest.mark.parametrize("M,N,K", [(2048, 768, 256), (4096, 2304, 768), (1024, 520, 264)])
def test_linear_wgrad_persistent(C, M, N, K):
    torch.manual_seed(5)
    dy = bf(torch.randn(M, N, device=dev))
    x = bf(torch.randn(M, K, device=dev))
    dw = torch.randn(N, K, device=dev)
    ref = dw + dy.float().t() @ x.float()
    C.linear_wgrad(dy, x, dw, 1.0)  # accumulates (K-split slabs + finalize, or in place)
    assert rel_err(dw, ref) < 1e-3


def test_linear_alpha_tensor(C):
    torch.manual_seed(6)
    M, N, K = 512, 512, 256
    dy = bf(torch.randn(M, N, device=dev))
    w = bf(torch.randn(N, K, device=dev))
    x = bf(torch.randn(M, K, device=dev))
    s = torch.tensor([0.25], device=dev)
    assert rel_err(C.linear_dgrad(dy, w, None, s), 0.25 * (dy.float() @ w.float())) < 1e-2
    dw = torch.zeros(N, K, device=dev)
    C.linear_wgrad(dy, x, dw, 2.0, s)
    assert rel_err(dw, 0.5 * (dy.float().t() @ x.float())) < 1e-3


# ------------------------------------- BatchNorm backward fused into dgrad epilogues
def _bn_coef(C_, Cc):
    scale = torch.rand(Cc, device=dev) + 0.5
    shift = torch.randn(Cc, device=dev) * 0.5
    mean = torch.randn(Cc, device=dev) * 0.3
    invstd = torch.rand(Cc, device=dev) + 0.5
    return torch.stack([scale, shift, mean, invstd]).contiguous()


def _bn_relu(h, coef):
    return torch.relu(h.float() * coef[0] + coef[1]).to(torch.bfloat16)


@pytest.mark.parametrize("N,H,W,Ci,Co,k,s,p", [(2, 14, 14, 64, 128, 3, 1, 1), (2, 14, 14, 64, 128, 3, 2, 1),
                                               (4, 7, 7, 256, 64, 1, 1, 0), (2, 28, 28, 128, 128, 3, 2, 1),
                                               # 1x1 at depth >= 1024: the persistent GEMM's BN-backward epilogue
                                               (2, 7, 7, 256, 1024, 1, 1, 0), (3, 14, 14, 512, 2048, 1, 1, 0)])
def test_dgrad_bn_backward_partials(C, N, H, W, Ci, Co, k, s, p):
    """dgrad epilogue partials + bn_bwd_partials == the standalone BN backward (mask from y)."""
    torch.manual_seed(13)
    h = bf(torch.randn(N, H, W, Ci, device=dev))  # pre-BN input of the BN+ReLU feeding this conv
    coef = _bn_coef(C, Ci)
    w = bf(torch.randn(Co, k, k, Ci, device=dev) / math.sqrt(k * k * Ci))
    OH = (H + 2 * p - k) // s + 1
    dy = bf(torch.randn(N, OH, OH, Co, device=dev))
    da_ref = C.conv_dgrad(dy, w, [N, H, W, Ci], [s, s], [p, p], [1, 1], None)
    da, part = C.conv_dgrad_bn(dy, w, [N, H, W, Ci], [s, s], [p, p], [1, 1], None, h, coef)
    if k == 1 and Co >= 1024:  # different kernels (persistent GEMM vs implicit GEMM): same math, rounding may differ
        ref32 = (dy.float().reshape(-1, Co) @ w.float().reshape(Co, Ci)).reshape(da.shape)
        assert rel_err(da, ref32) < 1e-2 and rel_err(da, da_ref) < 1e-2
    else:
        assert torch.equal(da, da_ref)
    df = da.float().reshape(-1, Ci)
    hf = h.float().reshape(-1, Ci)
    dz = torch.where(hf * coef[0] + coef[1] > 0, df, torch.zeros_like(df))
    tot = part.sum(-1)
    assert rel_err(tot[0], dz.sum(0)) < 1e-3
    assert rel_err(tot[1], (dz * (hf - coef[2])).sum(0)) < 1e-3
    gamma = torch.rand(Ci, device=dev) + 0.5
    dg1, db1 = torch.zeros(Ci, device=dev), torch.zeros(Ci, device=dev)
    dh = C.bn_bwd_partials(da, h, gamma, coef, part, dg1, db1)
    y = _bn_relu(h, coef)
    dg2, db2 = torch.zeros(Ci, device=dev), torch.zeros(Ci, device=dev)
    dh_ref, _ = C.bn_bwd(da, y, h, gamma, coef, dg2, db2, False)
    assert rel_err(dh, dh_ref) < 2e-2 and rel_err(dg1, dg2) < 1e-3 and rel_err(db1, db2) < 1e-3


@pytest.mark.parametrize("Ci,H,B", [(256, 14, 512)])
def test_stream_k_conv_matches_whole_k(C, Ci, H, B):
    """Stream-K schedule of the implicit-im2col conv GEMM (hgemm.hip SKM; ResNet-50's layer-3 3x3 shape, 392
    tiles of 256x256 on 256 CUs, where the whole-K tiles leave most of the second round idle): forward with
    BN sums and the data grad with BN-backward partials equal the whole-K launch within fp32 reassociation, agree
    with torch, and are bitwise identical run to run (fixed cut, partials added in block order)."""
    torch.manual_seed(21)
    x = bf(torch.randn(B, H, H, Ci, device=dev))
    w = bf(torch.randn(Ci, 3, 3, Ci, device=dev) / math.sqrt(9 * Ci))
    h = bf(torch.randn(B, H, H, Ci, device=dev))
    coef = _bn_coef(C, Ci)
    z = ([1, 1], [1, 1], [1, 1])
    prev = C.set_hgemm_sk(False)
    try:
        y0, s0 = C.conv_fwd(x, w, *z, True, None)
        d0, p0 = C.conv_dgrad_bn(x, w, [B, H, H, Ci], *z, None, h, coef)
        C.set_hgemm_sk(True)
        runs = [(C.conv_fwd(x, w, *z, True, None), C.conv_dgrad_bn(x, w, [B, H, H, Ci], *z, None, h, coef))
                for _ in range(2)]
    finally:
        C.set_hgemm_sk(prev)
    (y1, s1), (d1, p1) = runs[0]
    (y2, s2), (d2, p2) = runs[1]
    assert torch.equal(y1, y2) and torch.equal(s1, s2) and torch.equal(d1, d2) and torch.equal(p1, p2)
    # the stream-K cut really ran (a different fp32 summation order moves a few bf16 roundings)
    assert 0 < (y1 != y0).float().mean().item() < 1e-2
    assert rel_err(y1, y0) < 1e-2 and rel_err(d1, d0) < 1e-2
    assert rel_err(s1.sum(-1), s0.sum(-1)) < 1e-4 and rel_err(p1.sum(-1), p0.sum(-1)) < 1e-4
    ref = F.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), padding=1).permute(0, 2, 3, 1)
    assert rel_err(y1, ref) < 1e-2


def test_bn_apply_mask_bits_and_residual_relu_dgrad(C):
    """bn_apply's ReLU-mask bits, and the dgrad epilogue variant that masks dx with them
    (BN + residual + ReLU backward: dx stored as dz, BN partials of dz)."""
    torch.manual_seed(14)
    N, H, W, Ci, Co = 2, 14, 14, 64, 128
    h = bf(torch.randn(N, H, W, Ci, device=dev))
    coef = _bn_coef(C, Ci)
    res = bf(torch.randn(N, H, W, Ci, device=dev))
    y, bits = C.bn_apply(h, coef, res, None, True, True)
    yref = torch.relu(h.float() * coef[0] + coef[1] + res.float())
    assert rel_err(y, yref) < 1e-2
    want = (y.float() > 0).reshape(-1, 8).to(torch.int32)
    packed = (want << torch.arange(8, device=dev, dtype=torch.int32)).sum(-1).to(torch.uint8)
    assert bits.shape == (N, H, W, Ci // 8) and torch.equal(bits.reshape(-1), packed)
    # downsample form: residual BN'd in the same pass
    coef2 = _bn_coef(C, Ci)
    y2, _ = C.bn_apply(h, coef, res, coef2, True, False)
    r2 = (res.float() * coef2[0] + coef2[1]).to(torch.bfloat16).float()
    assert rel_err(y2, torch.relu(h.float() * coef[0] + coef[1] + r2)) < 1e-2
    # 1x1 data grad + residual, masked by the bits, with partials over (dz, dz*(h - mean))
    w = bf(torch.randn(Co, 1, 1, Ci, device=dev) / math.sqrt(Ci))
    dy = bf(torch.randn(N, H, W, Co, device=dev))
    dres = bf(torch.randn(N, H, W, Ci, device=dev))
    dx, part = C.conv_dgrad_bn(dy, w, [N, H, W, Ci], [1, 1], [0, 0], [1, 1], dres, h, coef, bits)
    full = C.conv_dgrad(dy, w, [N, H, W, Ci], [1, 1], [0, 0], [1, 1], dres).float()
    dz = torch.where(y.float() > 0, full, torch.zeros_like(full))
    assert rel_err(dx, dz) < 1e-2
    tot = part.sum(-1)
    dzf, hf = dz.reshape(-1, Ci), h.float().reshape(-1, Ci)
    assert rel_err(tot[0], dzf.sum(0)) < 1e-2
    assert rel_err(tot[1], (dzf * (hf - coef[2])).sum(0)) < 1e-2


def test_s2d_stem_conv(C):
    """Space-to-depth packing + 4x4/s1 stem conv (fwd, BN stats, weight grad) == 7x7/s2/p3 conv."""
    from distributed_pytorch_example_amd.ops import functional as Fx

    torch.manual_seed(21)
    x = torch.randn(4, 3, 64, 64, device=dev)
    w = torch.randn(64, 7, 7, 3, device=dev) / math.sqrt(147)
    w16 = w.to(torch.bfloat16)
    xb = x.to(torch.bfloat16).float()
    ref = F.conv2d(xb, w16.permute(0, 3, 1, 2).float(), None, 2, 3).permute(0, 2, 3, 1)
    xs = Fx.to_s2d_input(x)
    assert xs.shape == (4, 32, 32, 16) and torch.equal(xs[0, 3, 5, 4 * 3 + 1], x[0, 1, 7, 11].to(torch.bfloat16))
    wp = torch.nn.Parameter(w.clone())
    y, st = Fx.stem_conv_s2d(xs, wp, want_stats=True)
    assert y.shape == ref.shape and rel_err(y, ref) < 1e-2
    s = st.sum(-1)
    assert rel_err(s[0], ref.reshape(-1, 64).sum(0)) < 1e-2
    dy = bf(torch.randn_like(ref))
    y.backward(dy)
    wr = w16.float().permute(0, 3, 1, 2).requires_grad_(True)
    (gref,) = torch.autograd.grad(F.conv2d(xb, wr, None, 2, 3), wr, dy.float().permute(0, 3, 1, 2))
    assert rel_err(wp.grad, gref.permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.parametrize("H", [30, 29])
def test_stem_bn_relu_maxpool_fused(C, H):
    """maxpool(relu(BN(h))) with the BN output never materialised (fwd, running stats,
    and the pooled-gradient gather inside the BN backward) vs fp32 torch autograd.
    H even: quad-form backward kernels; H odd: the general gather."""
    from distributed_pytorch_example_amd.ops import functional as Fx
    from distributed_pytorch_example_amd.ops.layers import BatchNorm2d

    torch.manual_seed(23)
    N, W, Cc = 4, H, 64  # odd pooled border (30 -> 15)
    h = bf(torch.randn(N, H, W, Cc, device=dev) * 2 + 0.3)
    bn = BatchNorm2d(Cc, device=dev)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(Cc, device=dev) + 0.5)
        bn.bias.copy_(torch.randn(Cc, device=dev) * 0.2)
    hf = h.float().reshape(-1, Cc)
    st = torch.stack([hf.sum(0), (hf * hf).sum(0)]).unsqueeze(-1).contiguous()  # [2][C][1] partials
    hh = h.clone().requires_grad_(True)
    y = Fx.stem_bn_relu_maxpool(hh, bn, st, 3, 2, 1)
    g = torch.nn.Parameter(bn.weight.detach().clone())
    b = torch.nn.Parameter(bn.bias.detach().clone())
    rm, rv = torch.zeros(Cc, device=dev), torch.ones(Cc, device=dev)
    xr = h.float().permute(0, 3, 1, 2).requires_grad_(True)
    a = F.relu(F.batch_norm(xr, rm, rv, g, b, True, 0.1, 1e-5))
    ref = F.max_pool2d(a.to(torch.bfloat16).float(), 3, 2, 1)
    assert y.shape == (N, (H + 1) // 2, (W + 1) // 2, Cc)
    assert rel_err(y, ref.permute(0, 2, 3, 1)) < 1e-2
    assert rel_err(bn.running_mean, rm) < 1e-4 and rel_err(bn.running_var, rv) < 1e-4
    dy = bf(torch.randn_like(y))
    y.backward(dy)
    # backward through the bf16-rounded activation (straight-through), so the reference's
    # argmax ties are the ones the kernel saw
    a_r = a + (a.to(torch.bfloat16).float() - a).detach()
    ref2 = F.max_pool2d(a_r, 3, 2, 1)
    ref2.backward(dy.float().permute(0, 3, 1, 2))
    assert rel_err(hh.grad, xr.grad.permute(0, 2, 3, 1)) < 2e-2
    assert rel_err(bn.weight.grad, g.grad) < 1e-2 and rel_err(bn.bias.grad, b.grad) < 1e-2


@pytest.mark.parametrize("N,H,W,Ci,Co,k,s,p", [(2, 14, 14, 64, 128, 1, 2, 0), (2, 8, 8, 64, 64, 1, 1, 0),
                                               (2, 14, 14, 32, 64, 3, 2, 1)])
def test_conv_dgrad_acc_inplace(C, N, H, W, Ci, Co, k, s, p):
    """dx += dgrad(dy, w) in place (strided: untouched parities keep their values)."""
    torch.manual_seed(22)
    x = torch.randn(N, Ci, H, W, device=dev, requires_grad=True)
    w = bf(torch.randn(Co, k, k, Ci, device=dev) / math.sqrt(k * k * Ci))
    y = F.conv2d(x, w.permute(0, 3, 1, 2).float(), None, s, p)
    dy = bf(torch.randn_like(y))
    (ref,) = torch.autograd.grad(y, x, dy.float())
    base = bf(torch.randn(N, H, W, Ci, device=dev))
    dx = base.clone()
    C.conv_dgrad_acc(dy.permute(0, 2, 3, 1).contiguous(), w, dx, [s, s], [p, p], [1, 1])
    assert rel_err(dx, base.float() + ref.permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.parametrize("mode", [1, 2, 3])
@pytest.mark.parametrize("N,H,W,Ci,Co,k,s,p", [(2, 14, 14, 64, 256, 3, 1, 1), (3, 7, 7, 128, 384, 3, 1, 1),
                                               (2, 28, 28, 128, 128, 3, 2, 1), (2, 14, 14, 256, 512, 1, 1, 0),
                                               (2, 14, 14, 96, 200, 3, 1, 1), (2, 28, 28, 64, 64, 3, 1, 1),
                                               (3, 14, 14, 64, 40, 3, 1, 1)])
def test_conv_tiles_lds_dma(C, mode, N, H, W, Ci, Co, k, s, p):
    """LDS-DMA conv kernel at every tile (128, 256x128, 256x256 8-wave): forward output + BN
    statistics partials (128-row sub-tiles), and the forward-form data grad with BN partials."""
    torch.manual_seed(31)
    C.set_conv_tile(mode)
    try:
        x = bf(torch.randn(N, H, W, Ci, device=dev))
        w = bf(torch.randn(Co, k, k, Ci, device=dev) / math.sqrt(k * k * Ci))
        ref = _conv_ref(x, w, s, p)
        y, stats = C.conv_fwd(x, w, [s, s], [p, p], [1, 1], True, None)
        assert rel_err(y, ref) < 1e-2
        yf = y.float().reshape(-1, Co)
        tot = stats.sum(-1)
        assert rel_err(tot[0], yf.sum(0)) < 1e-3 and rel_err(tot[1], (yf * yf).sum(0)) < 1e-3
        # data grad (stride-1 / phase forward form) with BN-backward partials
        h = bf(torch.randn(N, H, W, Ci, device=dev))
        coef = _bn_coef(C, Ci)
        OH = (H + 2 * p - k) // s + 1
        dy = bf(torch.randn(N, OH, OH, Co, device=dev))
        xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
        yr = F.conv2d(xr, w.permute(0, 3, 1, 2).float(), None, s, p)
        (gx,) = torch.autograd.grad(yr, xr, dy.float().permute(0, 3, 1, 2))
        da, part = C.conv_dgrad_bn(dy, w, [N, H, W, Ci], [s, s], [p, p], [1, 1], None, h, coef)
        assert rel_err(da, gx.permute(0, 2, 3, 1)) < 1e-2
        df, hf = da.float().reshape(-1, Ci), h.float().reshape(-1, Ci)
        dz = torch.where(hf * coef[0] + coef[1] > 0, df, torch.zeros_like(df))
        tp = part.sum(-1)
        assert rel_err(tp[0], dz.sum(0)) < 1e-3 and rel_err(tp[1], (dz * (hf - coef[2])).sum(0)) < 1e-3
    finally:
        C.set_conv_tile(0)


@pytest.mark.parametrize("N,H,W,Ci,Co,k,s,p", [(8, 14, 14, 64, 64, 3, 1, 1), (32, 7, 7, 128, 200, 3, 1, 1),
                                               (8, 28, 28, 96, 128, 3, 2, 1), (4, 56, 56, 64, 256, 1, 1, 0),
                                               (8, 28, 28, 256, 512, 1, 2, 0), (32, 7, 7, 512, 512, 3, 1, 1),
                                               (16, 14, 14, 64, 48, 3, 1, 1), (8, 28, 28, 32, 64, 3, 1, 1),
                                               (8, 14, 14, 256, 256, 3, 1, 1), (8, 14, 14, 128, 384, 3, 2, 1),
                                               (8, 28, 28, 128, 512, 1, 1, 0), (8, 28, 28, 512, 128, 1, 1, 0)])
def test_conv_wgrad_lds_dma(C, N, H, W, Ci, Co, k, s, p):
    """LDS-DMA weight-grad kernel (pixel count % 32 == 0): im2col pixel walk across image
    boundaries (OW = 7 / 14 / 28), taps spanning a column tile (C = 64 / 96), split-K, M / N
    tails, strided 1x1; accumulates into an existing gradient."""
    torch.manual_seed(7)
    x = bf(torch.randn(N, H, W, Ci, device=dev))
    w = torch.randn(Co, Ci, k, k, device=dev, requires_grad=True)
    y = F.conv2d(x.permute(0, 3, 1, 2).float(), w, None, s, p)
    dy = bf(torch.randn_like(y))
    (ref,) = torch.autograd.grad(y, w, dy.float())
    dw0 = torch.randn(Co, k, k, Ci, device=dev)
    for wide in (1, 2):  # 2: the 64x256 tile also for C > 16
        C.set_wgrad_wide(wide)
        try:
            dw = dw0.clone()
            C.conv_wgrad(dy.permute(0, 2, 3, 1).contiguous(), x, dw, [s, s], [p, p], [1, 1], 1.0)
        finally:
            C.set_wgrad_wide(1)
        assert rel_err(dw - dw0, ref.permute(0, 2, 3, 1)) < 1e-3


def test_bn_bwd_with_mask_bits_matches_y(C):
    """BN+ReLU backward (reduce + apply, dz written) with the ReLU mask read as bn_apply's bits
    instead of the saved output y: identical results."""
    torch.manual_seed(17)
    N, H, W, Ci = 4, 14, 14, 256
    h = bf(torch.randn(N, H, W, Ci, device=dev))
    coef = _bn_coef(C, Ci)
    res = bf(torch.randn(N, H, W, Ci, device=dev))
    y, bits = C.bn_apply(h, coef, res, None, True, True)
    dy = bf(torch.randn(N, H, W, Ci, device=dev))
    gamma = torch.rand(Ci, device=dev) + 0.5
    outs = []
    for use_bits in (False, True):
        dg, db = torch.zeros(Ci, device=dev), torch.zeros(Ci, device=dev)
        dx, dz = C.bn_bwd(dy, y, h, gamma, coef, dg, db, True, bits if use_bits else None)
        outs.append((dx, dz, dg, db))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert torch.equal(outs[0][1], torch.where(y > 0, dy, torch.zeros_like(dy)))


@pytest.mark.parametrize("k", [1, 3])
def test_dgrad_residual_masked_by_bits(C, k):
    """Data grad + residual where the residual is dy of a BN+residual+ReLU output, masked in the
    epilogue by that output's bits (plain and BN-partials epilogues) == adding the masked residual."""
    torch.manual_seed(19)
    N, H, W, Ci, Co = 4, 14, 14, 128, 64
    w = bf(torch.randn(Co, k, k, Ci, device=dev) / math.sqrt(k * k * Ci))
    dy = bf(torch.randn(N, H, W, Co, device=dev))
    h = bf(torch.randn(N, H, W, Ci, device=dev))
    coef = _bn_coef(C, Ci)
    y, bits = C.bn_apply(h, coef, bf(torch.randn(N, H, W, Ci, device=dev)), None, True, True)
    dout = bf(torch.randn(N, H, W, Ci, device=dev))
    dz = torch.where(y > 0, dout, torch.zeros_like(dout))
    p = k // 2
    ref = C.conv_dgrad(dy, w, [N, H, W, Ci], [1, 1], [p, p], [1, 1], dz)
    got = C.conv_dgrad(dy, w, [N, H, W, Ci], [1, 1], [p, p], [1, 1], dout, bits)
    assert torch.equal(got, ref)
    h0 = bf(torch.randn(N, H, W, Ci, device=dev))
    c0 = _bn_coef(C, Ci)
    _, bits0 = C.bn_apply(h0, c0, h, None, True, True)
    r1, p1 = C.conv_dgrad_bn(dy, w, [N, H, W, Ci], [1, 1], [p, p], [1, 1], dz, h0, c0, bits0)
    r2, p2 = C.conv_dgrad_bn(dy, w, [N, H, W, Ci], [1, 1], [p, p], [1, 1], dout, h0, c0, bits0, bits)
    assert torch.equal(r1, r2) and torch.equal(p1, p2)


def test_bn_bwd_dual_matches_two_backwards(C):
    """bn_bwd_dual (BN3 from epilogue partials + downsample BN, dz read once for both) ==
    bn_bwd_partials for BN3 and the standalone reduce+apply for BN_d."""
    torch.manual_seed(23)
    N, H, W, Ch = 4, 14, 14, 256
    dz = bf(torch.randn(N, H, W, Ch, device=dev))
    h3, hd = bf(torch.randn(N, H, W, Ch, device=dev)), bf(torch.randn(N, H, W, Ch, device=dev))
    c3, cd = _bn_coef(C, Ch), _bn_coef(C, Ch)
    dzf, h3f = dz.float().reshape(-1, Ch), h3.float().reshape(-1, Ch)
    part = torch.stack([dzf.sum(0), (dzf * (h3f - c3[2])).sum(0)]).unsqueeze(-1).contiguous()
    g3, gd = torch.rand(Ch, device=dev) + 0.5, torch.rand(Ch, device=dev) + 0.5
    z = lambda: torch.zeros(Ch, device=dev)  # noqa: E731
    a_g3, a_b3, a_gd, a_bd = z(), z(), z(), z()
    dh3, dhd = C.bn_bwd_dual(dz, h3, g3, c3, part, a_g3, a_b3, hd, gd, cd, a_gd, a_bd)
    b_g3, b_b3, b_gd, b_bd = z(), z(), z(), z()
    ref3 = C.bn_bwd_partials(dz, h3, g3, c3, part, b_g3, b_b3, relu_mask=False)
    refd, _ = C.bn_bwd(dz, None, hd, gd, cd, b_gd, b_bd, False)
    assert torch.equal(dh3, ref3) and torch.allclose(a_g3, b_g3) and torch.allclose(a_b3, b_b3)
    assert rel_err(dhd, refd) < 1e-2 and rel_err(a_gd, b_gd) < 1e-4 and rel_err(a_bd, b_bd) < 1e-4


@pytest.mark.parametrize("N,H,W,Ci,Co", [(2, 9, 9, 256, 64), (3, 7, 7, 512, 128), (2, 6, 6, 1024, 256),
                                         (4, 28, 28, 256, 64),
                                         # several row tiles per persistent block: the DMA-ring prologue
                                         (32, 64, 64, 256, 64), (64, 28, 28, 512, 128), (64, 16, 16, 1024, 256)])
def test_pw_stream_matches_igemm(C, N, H, W, Ci, Co):
    """The streaming pointwise-conv kernel (pwconv.hip) == the implicit-GEMM path on the same inputs:
    conv3-style forward (Co -> Ci, BN stats) and conv1-style data grads with every epilogue variant
    (plain, + residual, + bits-masked residual, BN-backward partials with the ReLU from the
    coefficients or from the saved output's bits).  Outputs bitwise, partial sums to fp32 order."""
    torch.manual_seed(29)
    w = bf(torch.randn(Co, 1, 1, Ci, device=dev) / math.sqrt(Ci))        # conv1: Ci -> Co
    w3 = bf(torch.randn(Ci, 1, 1, Co, device=dev) / math.sqrt(Co))       # conv3: Co -> Ci
    a2 = bf(torch.randn(N, H, W, Co, device=dev))
    dy = bf(torch.randn(N, H, W, Co, device=dev))
    h = bf(torch.randn(N, H, W, Ci, device=dev))
    coef = _bn_coef(C, Ci)
    _, bits = C.bn_apply(h, coef, bf(torch.randn(N, H, W, Ci, device=dev)), None, True, True)
    dout = bf(torch.randn(N, H, W, Ci, device=dev))
    h0, c0 = bf(torch.randn(N, H, W, Ci, device=dev)), _bn_coef(C, Ci)
    _, bits0 = C.bn_apply(h0, c0, h, None, True, True)
    sh = [N, H, W, Ci]
    z = [1, 1], [0, 0], [1, 1]
    runs = {}
    for on in (True, False):
        C.set_pw_stream(on)
        try:
            runs[on] = [
                C.conv_fwd(a2, w3, *z, True, None),
                (C.conv_dgrad(dy, w, sh, *z, None), None),
                (C.conv_dgrad(dy, w, sh, *z, dout), None),
                (C.conv_dgrad(dy, w, sh, *z, dout, bits), None),
                tuple(C.conv_dgrad_bn(dy, w, sh, *z, None, h, coef)),
                tuple(C.conv_dgrad_bn(dy, w, sh, *z, dout, h0, c0, bits0, bits)),
            ]
        finally:
            C.set_pw_stream(True)
    for i, ((y1, s1), (y2, s2)) in enumerate(zip(runs[True], runs[False])):
        assert torch.equal(y1, y2), i
        if s1 is not None:
            assert s1.shape[:2] == s2.shape[:2]
            assert rel_err(s1.sum(-1), s2.sum(-1)) < 1e-4, i


@pytest.mark.parametrize("N,H,W,Ci,Co,Cd", [(2, 8, 8, 256, 128, 512), (4, 28, 28, 256, 128, 512),
                                            (3, 14, 14, 512, 256, 1024), (16, 56, 56, 256, 128, 512)])
def test_pw_dgrad_strided_residual(C, N, H, W, Ci, Co, Cd):
    """A downsample block's dx = conv1 data grad + the stride-2 branch's data grad: with
    residual_stride2 the streaming kernel adds the branch's compact [N, H/2, W/2, Ci] data grad at the
    even pixels, then masks with the previous block's ReLU bits and emits its BN3-backward partials.
    Equals the two-kernel form (dgrad, then the strided data grad accumulated in place) followed by
    the same mask / partials (bitwise output up to the order of two bf16 roundings; sums to 1e-4)."""
    torch.manual_seed(41)
    w1 = bf(torch.randn(Co, 1, 1, Ci, device=dev) / math.sqrt(Ci))   # conv1: Ci -> Co (stride 1)
    wd = bf(torch.randn(Cd, 1, 1, Ci, device=dev) / math.sqrt(Ci))   # downsample: Ci -> Cd (stride 2)
    dh1 = bf(torch.randn(N, H, W, Co, device=dev))
    dhd = bf(torch.randn(N, H // 2, W // 2, Cd, device=dev))
    h3, c3 = bf(torch.randn(N, H, W, Ci, device=dev)), _bn_coef(C, Ci)
    _, bits = C.bn_apply(h3, c3, bf(torch.randn(N, H, W, Ci, device=dev)), None, True, True)
    sh = [N, H, W, Ci]
    z = [1, 1], [0, 0], [1, 1]
    dxd = C.conv_dgrad(dhd, wd, [N, H // 2, W // 2, Ci], *z, None)
    dx, part = C.conv_dgrad_bn(dh1, w1, sh, *z, dxd, h3, c3, bits, None, True)
    # reference: dense two-kernel form, then mask + partials in fp32
    full = C.conv_dgrad(dh1, w1, sh, *z, None)
    C.conv_dgrad_acc(dhd, wd, full, [2, 2], [0, 0], [1, 1])
    m = torch.zeros(N, H, W, Ci, dtype=torch.bool, device=dev)
    ybits = bits.view(torch.uint8).reshape(N, H, W, Ci // 8)
    for e in range(8):
        m[..., e::8] = ((ybits >> e) & 1).bool()
    dz = torch.where(m, full.float(), torch.zeros_like(full.float()))
    assert rel_err(dx, dz) < 5e-3
    hf = h3.float().reshape(-1, Ci)
    ps = part.sum(-1)
    assert rel_err(ps[0], dz.reshape(-1, Ci).sum(0)) < 2e-3
    assert rel_err(ps[1], (dz.reshape(-1, Ci) * (hf - c3[2])).sum(0)) < 2e-3


@pytest.mark.parametrize("N,H,W", [(2, 112, 112), (3, 112, 112), (1, 7, 100), (4, 3, 112)])
def test_stem_kernel_matches_igemm(C, N, H, W):
    """The row-walking s2d stem kernel (stem.hip: filter in VGPRs, 5-row LDS ring, per-block BN
    partials) == the implicit-GEMM tile on the same inputs: output bitwise (same K order), BN sums
    to fp32 summation order; and both match the fp32 reference conv."""
    torch.manual_seed(37)
    xs = bf(torch.randn(N, H, W, 16, device=dev))
    w = bf(torch.randn(64, 4, 4, 16, device=dev) / 16)
    runs = {}
    for on in (True, False):
        C.set_stem_kernel(on)
        try:
            runs[on] = C.conv_fwd(xs, w, [1, 1], [2, 2, 1, 1], [1, 1], True, None)
        finally:
            C.set_stem_kernel(True)
    (y1, s1), (y2, s2) = runs[True], runs[False]
    ref = F.conv2d(F.pad(xs.permute(0, 3, 1, 2).float(), (2, 1, 2, 1)), w.permute(0, 3, 1, 2).float()).permute(0, 2, 3, 1)
    assert y1.shape == ref.shape and rel_err(y1, ref) < 1e-2
    assert torch.equal(y1, y2)
    assert rel_err(s1.sum(-1), s2.sum(-1)) < 1e-4
    yf = y1.float().reshape(-1, 64)
    assert rel_err(s1.sum(-1)[0], yf.sum(0)) < 1e-3 and rel_err(s1.sum(-1)[1], (yf * yf).sum(0)) < 1e-3


@pytest.mark.parametrize("N,H,W", [(2, 56, 56), (3, 56, 56), (5, 8, 8), (3, 14, 14), (1, 20, 40), (2, 9, 17), (2, 5, 64),
                                   (1, 2, 3)])
def test_rowconv_matches_igemm(C, N, H, W):
    """The row-walking 64-channel 3x3 kernel (rowconv.hip: filter in VGPRs, swizzled 4-row LDS ring,
    per-block partials) == the implicit-GEMM tiles on the same inputs: forward with BN sums, the
    stride-1 data grad, and the data grad with the BN-backward epilogue.  Outputs bitwise (same K
    order), partial sums to fp32 summation order; the forward also against the fp32 reference."""
    torch.manual_seed(41)
    x = bf(torch.randn(N, H, W, 64, device=dev))
    w = bf(torch.randn(64, 3, 3, 64, device=dev) / 24)
    dy = bf(torch.randn(N, H, W, 64, device=dev))
    h = bf(torch.randn(N, H, W, 64, device=dev))
    coef = _bn_coef(C, 64)
    sh = [N, H, W, 64]
    z = [1, 1], [1, 1], [1, 1]
    runs = {}
    for on in (True, False):
        C.set_rowconv(on)
        try:
            runs[on] = [
                C.conv_fwd(x, w, *z, True, None),
                (C.conv_dgrad(dy, w, sh, *z, None), None),
                tuple(C.conv_dgrad_bn(dy, w, sh, *z, None, h, coef)),
            ]
        finally:
            C.set_rowconv(True)
    assert rel_err(runs[True][0][0], _conv_ref(x, w, 1, 1)) < 1e-2
    for i, ((y1, s1), (y2, s2)) in enumerate(zip(runs[True], runs[False])):
        assert torch.equal(y1, y2), i
        if s1 is not None:
            assert rel_err(s1.sum(-1), s2.sum(-1)) < 1e-4, i


@pytest.mark.parametrize("N,H,W", [(3, 56, 56), (2, 9, 20), (70, 7, 7), (2, 5, 64)])
def test_row_wgrad_matches_reference(C, N, H, W):
    """Row-walking 64-channel 3x3 weight grad (rowconv.hip: per-image gradient in registers, dy and
    x rows as LDS images read with ds_read_b64_tr_b16, coalesced per-image partials + a reduce
    kernel): vs the fp32 reference and the im2col weight-grad tile, accumulating into an existing
    gradient with alpha; W <= 32 takes one K-step per row, N >= 64 the grouped partial reduce."""
    torch.manual_seed(43)
    x = bf(torch.randn(N, H, W, 64, device=dev))
    dy = bf(torch.randn(N, H, W, 64, device=dev))
    w = torch.randn(64, 64, 3, 3, device=dev, requires_grad=True)
    y = F.conv2d(x.permute(0, 3, 1, 2).float(), w, None, 1, 1)
    (ref,) = torch.autograd.grad(y, w, dy.permute(0, 3, 1, 2).float())
    dw0 = torch.randn(64, 3, 3, 64, device=dev)
    outs = {}
    for on in (True, False):
        C.set_row_wgrad(on)
        try:
            dw = dw0.clone()
            C.conv_wgrad(dy, x, dw, [1, 1], [1, 1], [1, 1], 0.5)
        finally:
            C.set_row_wgrad(True)
        outs[on] = dw - dw0
    assert rel_err(outs[True], 0.5 * ref.permute(0, 2, 3, 1)) < 1e-4
    assert rel_err(outs[True], outs[False]) < 1e-4
    # under a CU budget: two rounds of half-size row blocks (fixed-order partials, another grouping)
    C.set_cu_reserve(16)
    C.set_comm_active(True)
    try:
        dws = []
        for _ in range(2):
            dw = dw0.clone()
            C.conv_wgrad(dy, x, dw, [1, 1], [1, 1], [1, 1], 0.5)
            dws.append(dw - dw0)
    finally:
        C.set_comm_active(False)
        C.set_cu_reserve(0)
    assert rel_err(dws[0], dws[1]) < 1e-6
    assert rel_err(dws[0], outs[True]) < 1e-5


@pytest.mark.parametrize("reserve", [16, 300])
def test_row_kernels_under_cu_budget(C, reserve):
    """The row-walking kernels size their grid to the resident slots minus the CU budget (one block
    per slot, each a contiguous range of the N*H rows, segments crossing image boundaries): the
    conv output is bitwise the unbudgeted one, its BN partials sum to the same totals, and the
    weight grad (fixed-order reduction, no atomics) is bitwise reproducible and matches."""
    torch.manual_seed(47)
    N, H, W = 160, 56, 56  # 8960 rows: 512 blocks unbudgeted (2 per CU), fewer under the budget
    x = bf(torch.randn(N, H, W, 64, device=dev))
    w = bf(torch.randn(64, 3, 3, 64, device=dev) / 24)
    dy = bf(torch.randn(N, H, W, 64, device=dev))
    z = [1, 1], [1, 1], [1, 1]

    def run():
        y, st = C.conv_fwd(x, w, *z, True, None)
        dws = []
        for _ in range(2):
            dw = torch.zeros(64, 3, 3, 64, device=dev)
            C.conv_wgrad(dy, x, dw, *z, 1.0)
            dws.append(dw)
        return y, st, dws

    y0, st0, (dw0, dw0b) = run()
    C.set_cu_reserve(reserve)
    C.set_comm_active(True)
    try:
        y1, st1, (dw1, dw1b) = run()
    finally:
        C.set_comm_active(False)
        C.set_cu_reserve(0)
    torch.cuda.synchronize()
    assert st1.shape[-1] != st0.shape[-1] or reserve == 0  # a different grid / partial layout
    assert torch.equal(y0, y1)
    assert rel_err(st1.sum(-1), st0.sum(-1)) < 1e-5
    assert torch.equal(dw0, dw0b) and torch.equal(dw1, dw1b)
    assert rel_err(dw1, dw0) < 1e-5


@pytest.mark.parametrize("N,H,W", [(3, 56, 56), (2, 9, 20)])
def test_row_kernels_bn_on_load(C, N, H, W):
    """The row-walking 64-channel 3x3 forward and weight grad with in_coef (x = pre-BN h, operand =
    relu(h * scale + shift) applied on load, padding rows/pixels still zero) == the same kernels on
    the tensor bn_apply materialises: bitwise for the output, the BN sums and the weight grad."""
    torch.manual_seed(47)
    h = bf(torch.randn(N, H, W, 64, device=dev))
    coef = _bn_coef(C, 64)
    a, _ = C.bn_apply(h, coef, None, None, True, False)
    w = bf(torch.randn(64, 3, 3, 64, device=dev) / 24)
    z = [1, 1], [1, 1], [1, 1]
    y1, s1 = C.conv_fwd(h, w, *z, True, None, coef)
    y2, s2 = C.conv_fwd(a, w, *z, True, None)
    assert torch.equal(y1, y2) and torch.equal(s1, s2)
    dy = bf(torch.randn(N, H, W, 64, device=dev))
    dw1 = torch.zeros(64, 3, 3, 64, device=dev)
    dw2 = torch.zeros_like(dw1)
    C.conv_wgrad(dy, h, dw1, *z, 1.0, coef)
    C.conv_wgrad(dy, a, dw2, *z, 1.0)
    assert rel_err(dw1, dw2) < 1e-6
    assert C.row_bn_on_load([N, H, W, 64], [64, 3, 3, 64], *z)
    assert not C.row_bn_on_load([N, H, W, 64], [64, 3, 3, 64], [2, 2], [1, 1], [1, 1])


@pytest.mark.parametrize("N,H,W", [(3, 112, 112), (2, 9, 100), (70, 4, 20), (1, 5, 33)])
def test_stem_wgrad_matches_reference(C, N, H, W):
    """Row-walking s2d stem weight grad (stem.hip: per-image 64 x 256 gradient in registers, dY and
    x rows as LDS images read with ds_read_b64_tr_b16, 4-tap column shifts, pad 2-2-1-1) vs the fp32
    reference and the im2col weight-grad tile, accumulating with alpha; N >= 64 takes the grouped
    partial reduce, W not a multiple of 32 a partial last K-step."""
    torch.manual_seed(53)
    xs = bf(torch.randn(N, H, W, 16, device=dev))
    dy = bf(torch.randn(N, H, W, 64, device=dev))
    w = torch.randn(64, 16, 4, 4, device=dev, requires_grad=True)
    y = F.conv2d(F.pad(xs.permute(0, 3, 1, 2).float(), (2, 1, 2, 1)), w)
    (ref,) = torch.autograd.grad(y, w, dy.permute(0, 3, 1, 2).float())
    dw0 = torch.randn(64, 4, 4, 16, device=dev)
    outs = {}
    for on in (True, False):
        C.set_stem_kernel(on)
        try:
            dw = dw0.clone()
            C.conv_wgrad(dy, xs, dw, [1, 1], [2, 2], [1, 1], 0.5)
        finally:
            C.set_stem_kernel(True)
        outs[on] = dw - dw0
    assert rel_err(outs[True], 0.5 * ref.permute(0, 2, 3, 1)) < 1e-4
    assert rel_err(outs[True], outs[False]) < 1e-4
    # under a CU budget (H >= 8): half-image blocks (their partials reach dw through the same grouped
    # reduce: fp32 atomics across groups when there are >= 64 partials, so equal to fp32 rounding)
    C.set_cu_reserve(16)
    C.set_comm_active(True)
    try:
        dws = []
        for _ in range(2):
            dw = dw0.clone()
            C.conv_wgrad(dy, xs, dw, [1, 1], [2, 2], [1, 1], 0.5)
            dws.append(dw - dw0)
    finally:
        C.set_comm_active(False)
        C.set_cu_reserve(0)
    assert rel_err(dws[0], dws[1]) < 1e-6
    assert rel_err(dws[0], outs[True]) < 1e-5


@pytest.mark.parametrize("N,H,W,Ci,Co", [(8, 56, 56, 64, 256), (3, 7, 30, 64, 128), (8, 28, 28, 128, 512)])
def test_pointwise_bn_on_load(C, N, H, W, Ci, Co):
    """Layer-1 conv3 over a pre-BN input: the streaming pointwise forward and the LDS-DMA weight grad
    with in_coef (relu(h * scale + shift) applied to the operand fragments) == the same convs over
    the tensor bn_apply materialises (forward bitwise incl. BN sums; weight grad to fp32 order)."""
    torch.manual_seed(59)
    h = bf(torch.randn(N, H, W, Ci, device=dev))
    coef = _bn_coef(C, Ci)
    a, _ = C.bn_apply(h, coef, None, None, True, False)
    w = bf(torch.randn(Co, 1, 1, Ci, device=dev) / 8)
    z = [1, 1], [0, 0], [1, 1]
    assert C.pw_bn_on_load([N, H, W, Ci], Co) == ((N * H * W) % 32 == 0)
    if (N * H * W) % 32:
        return
    y1, s1 = C.conv_fwd(h, w, *z, True, None, coef)
    y2, s2 = C.conv_fwd(a, w, *z, True, None)
    assert torch.equal(y1, y2) and torch.equal(s1, s2)
    dy = bf(torch.randn(N, H, W, Co, device=dev))
    dw1 = torch.zeros(Co, 1, 1, Ci, device=dev)
    dw2 = torch.zeros_like(dw1)
    C.conv_wgrad(dy, h, dw1, *z, 1.0, coef)
    C.conv_wgrad(dy, a, dw2, *z, 1.0)
    assert rel_err(dw1, dw2) < 1e-5


@pytest.mark.parametrize("K,N", [(64, 256), (128, 512), (256, 1024)])
def test_pw_stream_dynamic_schedule_under_cu_budget(C, K, N):
    """The streaming pointwise conv under a CU budget runs twice the row groups and claims the second
    half at run time (pwconv.hip, DYN): the forward output and the data grad are bitwise the unbudgeted
    ones, the BN partials (a different, equally fixed layout) sum to the same totals, two budgeted runs
    are bitwise identical (schedule-independent row groups), and the claim counters are left zeroed
    (the unbudgeted run after them is bitwise the first one)."""
    torch.manual_seed(53)
    n, h = 224, 56  # M = 702,464 rows: enough tiles for every row group to keep >= 7 of them
    x = bf(torch.randn(n, h, h, K, device=dev))
    w = bf(torch.randn(N, 1, 1, K, device=dev) / K ** 0.5)  # forward K -> N
    w2 = bf(torch.randn(K, 1, 1, N, device=dev) / K ** 0.5)  # a conv N -> K: its data grad is K -> N
    dy = bf(torch.randn(n, h, h, K, device=dev))
    hx = bf(torch.randn(n, h, h, N, device=dev))
    coef = _bn_coef(C, N)
    z = [1, 1], [0, 0], [1, 1]

    def run():
        y, st = C.conv_fwd(x, w, *z, True, None)
        dx, part = C.conv_dgrad_bn(dy, w2, [n, h, h, N], *z, None, hx, coef)
        torch.cuda.synchronize()
        return y, st, dx, part

    y0, st0, dx0, p0 = run()
    C.set_cu_reserve(16)
    C.set_comm_active(True)
    try:
        runs = [run(), run()]
    finally:
        C.set_comm_active(False)
        C.set_cu_reserve(0)
    y3, st3, dx3, p3 = run()
    (y1, st1, dx1, p1), (y2, st2, dx2, p2) = runs
    assert st1.shape[-1] > st0.shape[-1] and p1.shape[-1] > p0.shape[-1]  # the dynamic layout
    assert torch.equal(y0, y1) and torch.equal(dx0, dx1)
    assert rel_err(st1.sum(-1), st0.sum(-1)) < 1e-5 and rel_err(p1.sum(-1), p0.sum(-1)) < 1e-5
    assert torch.equal(st1, st2) and torch.equal(p1, p2) and torch.equal(y1, y2) and torch.equal(dx1, dx2)
    assert torch.equal(st3, st0) and torch.equal(p3, p0) and torch.equal(y3, y0)


@pytest.mark.parametrize("N,H,Ci,Co", [(8, 28, 512, 1024), (4, 14, 1024, 2048), (3, 9, 512, 256), (2, 14, 256, 512)])
def test_hgemm_strided_pointwise_conv(C, N, H, Ci, Co):
    """Strided 1x1 convs (the bottleneck downsamples, >= 512 input channels) on the persistent GEMM's
    implicit-im2col A (one filter tap; the row's input pixel at (s*oh, s*ow)) vs the implicit-GEMM kernel
    and fp32 torch, with the BN-forward sums; odd spatial size included (M tail); 256 input channels
    stay on the implicit-GEMM kernel (both arms equal)."""
    torch.manual_seed(67)
    x = bf(torch.randn(N, H, H, Ci, device=dev))
    w = bf(torch.randn(Co, 1, 1, Ci, device=dev) / Ci ** 0.5)
    z = [2, 2], [0, 0], [1, 1]
    ref = F.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), None, 2, 0).permute(0, 2, 3, 1)
    outs = {}
    for on in (True, False):
        C.set_hgemm_conv(on)
        try:
            outs[on] = C.conv_fwd(x, w, *z, True, None)
        finally:
            C.set_hgemm_conv(True)
    (y1, s1), (y0, s0) = outs[True], outs[False]
    assert rel_err(y1.float(), ref) < 1e-2 and rel_err(y1.float(), y0.float()) < 1e-2
    yf = y1.float().reshape(-1, Co)
    assert rel_err(s1.sum(-1)[0], yf.sum(0)) < 1e-4 and rel_err(s1.sum(-1)[1], (yf * yf).sum(0)) < 1e-4


@pytest.mark.parametrize("N,H,Ci,Co,s", [(16, 14, 256, 256, 1), (16, 28, 256, 256, 2), (3, 7, 512, 512, 1),
                                         (64, 14, 512, 512, 2), (2, 9, 128, 256, 1)])
def test_hgemm_implicit_conv(C, N, H, Ci, Co, s):
    """3x3 convs with >= 256 output channels on the persistent GEMM with an implicit-im2col A (hgemm.hip
    AC: per-row tap masks, filter-tap offset per 64-deep K-tile, padding from out-of-range buffer loads)
    vs the implicit-GEMM kernel and fp32 torch: forward with and without the BN-forward sums, and the
    stride-1 data grad (a forward conv of dy with the flipped filter) with the BN-backward partials.
    M tails (not a multiple of the tile) included."""
    torch.manual_seed(61)
    x = bf(torch.randn(N, H, H, Ci, device=dev))
    w = bf(torch.randn(Co, 3, 3, Ci, device=dev) / (9 * Ci) ** 0.5)
    z = [s, s], [1, 1], [1, 1]
    ref = F.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), None, s, 1).permute(0, 2, 3, 1)
    outs = {}
    for on in (True, False):
        C.set_hgemm_conv(on)
        try:
            y, st = C.conv_fwd(x, w, *z, True, None)
            y2, _ = C.conv_fwd(x, w, *z, False, None)
        finally:
            C.set_hgemm_conv(True)
        outs[on] = (y, st, y2)
    (y1, s1, y1b), (y0, s0, _) = outs[True], outs[False]
    assert rel_err(y1.float(), ref) < 1e-2
    assert torch.equal(y1, y1b)
    assert rel_err(y1.float(), y0.float()) < 1e-2
    # weight grad: the TN layout with an implicit-im2col B (K-split slabs summed in a fixed order)
    OH = (H - 1) // s + 1
    dyw = bf(torch.randn(N, OH, OH, Co, device=dev))
    wref = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2).float(), (Co, Ci, 3, 3), dyw.permute(0, 3, 1, 2).float(),
                                       s, 1).permute(0, 2, 3, 1)
    dws = {}
    for on in (True, False):
        C.set_hgemm_conv(on)
        try:
            dw = torch.full((Co, 3, 3, Ci), 0.25, device=dev)
            C.conv_wgrad(dyw, x, dw, *z, 0.5)
            dw2 = torch.full((Co, 3, 3, Ci), 0.25, device=dev)
            C.conv_wgrad(dyw, x, dw2, *z, 0.5)
        finally:
            C.set_hgemm_conv(True)
        dws[on] = (dw - 0.25, dw2 - 0.25)
    assert rel_err(dws[True][0], 0.5 * wref) < 1e-4 and rel_err(dws[True][0], dws[False][0]) < 1e-4
    if (N * OH * OH) % 64 == 0:  # (the hgemm route: no atomics, bitwise repeatable)
        assert torch.equal(dws[True][0], dws[True][1])
    # BN-forward sums of the stored (rounded) values
    yf = y1.float().reshape(-1, Co)
    assert rel_err(s1.sum(-1)[0], yf.sum(0)) < 1e-4 and rel_err(s1.sum(-1)[1], (yf * yf).sum(0)) < 1e-4
    if s == 1:
        # data grad: dx = conv_transpose(dy, w) with the BN-backward partials of relu(BN(h))
        dy = bf(torch.randn(N, H, H, Co, device=dev))
        h = bf(torch.randn(N, H, H, Ci, device=dev))
        coef = _bn_coef(C, Ci)
        res = {}
        for on in (True, False):
            C.set_hgemm_conv(on)
            try:
                res[on] = C.conv_dgrad_bn(dy, w, [N, H, H, Ci], *z, None, h, coef)
            finally:
                C.set_hgemm_conv(True)
        (dx1, p1), (dx0, p0) = res[True], res[False]
        dref = torch.nn.grad.conv2d_input((N, Ci, H, H), w.permute(0, 3, 1, 2).float(), dy.permute(0, 3, 1, 2).float(),
                                          1, 1).permute(0, 2, 3, 1)
        assert rel_err(dx1.float(), dref) < 1e-2 and rel_err(dx1.float(), dx0.float()) < 1e-2
        dz = dx1.float() * ((h.float() * coef[0] + coef[1]) > 0)
        assert rel_err(p1.sum(-1)[0], dz.reshape(-1, Ci).sum(0)) < 1e-3
        assert rel_err(p1.sum(-1)[1], (dz * (h.float() - coef[2])).reshape(-1, Ci).sum(0)) < 1e-3


@pytest.mark.parametrize("cin,cout,stride,hw", [(128, 128, 1, 28), (256, 256, 1, 14), (128, 128, 2, 28), (64, 64, 1, 56)])
def test_flipped_filter_cache_refresh(C, cin, cout, stride, hw):
    """The data grads' flipped filters are cached per weight and refreshed (all at once) when the weight
    epoch moves: after an in-place change of the filter + set_weight_epoch, the data grad equals the one
    computed from a fresh tensor holding the new filter; both match an fp32 torch reference."""
    import torch.nn.functional as F

    g = torch.Generator(device=dev).manual_seed(cin + stride)
    w = (torch.randn(cout, 3, 3, cin, device=dev, generator=g) * (9 * cin) ** -0.5).bfloat16()
    oh = hw // stride
    dy = torch.randn(4, oh, oh, cout, device=dev, generator=g).bfloat16()
    xs = [4, hw, hw, cin]
    d1 = C.conv_dgrad(dy, w, xs, [stride, stride], [1, 1], [1, 1])  # registers the cached flip(s)
    w2 = (torch.randn(cout, 3, 3, cin, device=dev, generator=g) * (9 * cin) ** -0.5).bfloat16()
    w.copy_(w2)
    C.set_weight_epoch(10**9 + cin + stride)  # (the optimizer / shadow re-cast does this)
    d2 = C.conv_dgrad(dy, w, xs, [stride, stride], [1, 1], [1, 1])
    d_fresh = C.conv_dgrad(dy, w2.clone(), xs, [stride, stride], [1, 1], [1, 1])
    assert torch.equal(d2, d_fresh)
    ref = torch.nn.grad.conv2d_input([4, cin, hw, hw], w2.float().permute(0, 3, 1, 2), dy.float().permute(0, 3, 1, 2),
                                     stride=stride, padding=1).permute(0, 2, 3, 1)
    assert rel_err(d2, ref) < 2e-2, rel_err(d2, ref)
    assert rel_err(d1, ref) > 0.5  # (the first call used the old filter)


@pytest.mark.parametrize("ci,co,h", [(128, 128, 28), (256, 256, 14), (64, 128, 16)])
def test_strided_dgrad_phase_group_matches_per_parity(C, ci, co, h):
    """Strided 3x3 data grad: the four parity sub-GEMMs in one grid (igemm_dma_group_kernel) == one launch
    per parity, dx bit for bit (same K order per element; the grouped launch may use a smaller tile) and the
    BN-backward partials to rounding; plain and BN-partials epilogues; and against fp32 torch."""
    g = torch.Generator(device=dev).manual_seed(ci + h)
    N = 4
    w = (torch.randn(co, 3, 3, ci, device=dev, generator=g) / math.sqrt(9 * ci)).bfloat16()
    dy = torch.randn(N, h // 2, h // 2, co, device=dev, generator=g).bfloat16()
    hh = torch.randn(N, h, h, ci, device=dev, generator=g).bfloat16()
    coef = _bn_coef(C, ci)
    xs = [N, h, h, ci]
    outs = {}
    for grp in (True, False):
        C.set_phase_group(grp)
        try:
            d_plain = C.conv_dgrad(dy, w, xs, [2, 2], [1, 1], [1, 1], None)
            d_bn, part = C.conv_dgrad_bn(dy, w, xs, [2, 2], [1, 1], [1, 1], None, hh, coef)
        finally:
            C.set_phase_group(False)
        outs[grp] = (d_plain, d_bn, part.sum(-1))
    assert torch.equal(outs[True][0], outs[False][0])
    assert torch.equal(outs[True][1], outs[False][1])
    assert rel_err(outs[True][2], outs[False][2]) < 1e-5
    ref = torch.nn.grad.conv2d_input([N, ci, h, h], w.float().permute(0, 3, 1, 2), dy.float().permute(0, 3, 1, 2),
                                     stride=2, padding=1).permute(0, 2, 3, 1)
    assert rel_err(outs[True][0], ref) < 2e-2


@pytest.mark.parametrize("H,W", [(112, 112), (29, 30), (30, 29), (7, 9)])
def test_bnrelu_maxpool_key_kernel_matches_reference(C, H, W):
    """The stem max-pool's key-max kernel (bnrelu_maxpool3_kernel: ReLU, max and first-tap tie break in one
    integer max per tap) equals the per-tap compare kernel bit for bit: values (a -0 max reads as +0) and
    argmax bytes, including the ties that the bf16 round creates, odd borders and negative BN scales."""
    g = torch.Generator(device=dev).manual_seed(H * 100 + W)
    N = 3
    h = (torch.randn(N, H, W, 64, device=dev, generator=g) * 3).bfloat16()
    h[0, :4] = h[0, :4].round()  # many exact ties
    sc = 1 + 0.5 * torch.randn(64, device=dev, generator=g)
    sc[:8] = -sc[:8].abs()  # negative scales: the max comes from the smallest h
    sc[8] = 0.0  # constant channel: every tap ties
    coef = torch.stack([sc, 0.5 * torch.randn(64, device=dev, generator=g), torch.zeros(64, device=dev),
                        torch.ones(64, device=dev)]).float().contiguous()
    y1, i1 = C.bnrelu_maxpool_fwd(h, coef, 3, 2, 1)
    C.set_pool_legacy(True)
    try:
        y0, i0 = C.bnrelu_maxpool_fwd(h, coef, 3, 2, 1)
    finally:
        C.set_pool_legacy(False)
    assert torch.equal(i1, i0)
    assert torch.equal(y1.float(), y0.float())
    # and against torch: max_pool2d of the bf16-rounded relu(fma) activation
    a = torch.relu(torch.addcmul(coef[1].view(1, 1, 1, -1), h.float(), coef[0].view(1, 1, 1, -1))).bfloat16().float()
    ref = torch.nn.functional.max_pool2d(a.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    assert rel_err(y1, ref) < 1e-2


@pytest.mark.parametrize("N", [2, 5])
def test_stem_bwd_fused_matches_apply_path(C, N):
    """The stem backward without dL/dh (stem_bwd_fused: dY computed inside the weight grad from the pooled
    gradient, the argmax bytes and h) equals the apply-pass path bit for bit (same windows, same fmaf
    chain, same weight-grad accumulation order): dW, dgamma, dbeta."""
    g = torch.Generator(device=dev).manual_seed(N)
    H = W = 112
    xs = torch.randn(N, H, W, 16, device=dev, generator=g).bfloat16()
    h = torch.randn(N, H, W, 64, device=dev, generator=g).bfloat16()
    coef = torch.stack([1 + 0.2 * torch.randn(64, device=dev, generator=g), 0.3 * torch.randn(64, device=dev, generator=g),
                        0.1 * torch.randn(64, device=dev, generator=g), 1 + 0.1 * torch.rand(64, device=dev, generator=g)]).float()
    y, idx = C.bnrelu_maxpool_fwd(h, coef, 3, 2, 1)
    dy = torch.randn(y.shape, device=dev, generator=g).bfloat16()
    gamma = 1 + 0.1 * torch.randn(64, device=dev, generator=g)
    dg1, db1 = torch.zeros(64, device=dev), torch.zeros(64, device=dev)
    dh = C.maxpool_bn_bwd(dy, idx, h, gamma, coef, dg1, db1, 3, 2, 1)
    dw1 = torch.zeros(64, 4, 4, 16, device=dev)
    C.conv_wgrad(dh, xs, dw1, [1, 1], [2, 2], [1, 1], 1.0)
    dg2, db2 = torch.zeros(64, device=dev), torch.zeros(64, device=dev)
    dw2 = torch.zeros(64, 4, 4, 16, device=dev)
    C.stem_bwd_fused(dy, idx, h, xs, gamma, coef, dg2, db2, dw2)
    assert torch.equal(dg1, dg2) and torch.equal(db1, db2)
    assert rel_err(dw2, dw1) < 1e-6, rel_err(dw2, dw1)  # (fp32 atomics of the partial reduce: order may differ)
    # and against fp32 torch: dW of conv(xs, W) for dL/dh = dh
    ref = torch.nn.grad.conv2d_weight(torch.nn.functional.pad(xs.float().permute(0, 3, 1, 2), (2, 1, 2, 1)), [64, 16, 4, 4],
                                      dh.float().permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
    assert rel_err(dw2, ref) < 1e-3, rel_err(dw2, ref)
