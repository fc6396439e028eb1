"""BN3 by Gram algebra in the regime where E[h^2] - mean^2 cancels (VERDICT r4 missing #5 / next #6).

The Gram path never forms h3 = a2 W3^T: BN3's variance comes from w^T G w / M - mean^2 and the backward's
sum dz (h - mean) from w . P - mean sum dz.  Both cancel catastrophically when a channel's |mean| / std is
large, which trained networks reach (post-ReLU operands are non-negative, so a2 has a large common-mode
part).  Layer-1 scale (M = 512 * 56 * 56 rows, Cin = 64, Cout = 256), every h3 channel at |mean| / std >= 30;
the PER-CHANNEL relative error of the variance, of dgamma (= invstd * sum dz (h - mean); relative to the
larger of its value and the sum's natural magnitude, since a random-sign sum can land near zero) and of
the dW3 rows against an fp64 reference of the same bf16 operands must each stay below 1e-3.  Before the
centred Gram pass (bngram.hip relu_gauss_mean) the variance error was 2.2e-3 at |mean|/std = 177.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from distributed_pytorch_example_amd.ops._ext import ext  # noqa: E402

DEV = "cuda"


def _case(C, Cout, N, HW, seed, shift_level):
    g = torch.Generator(device=DEV).manual_seed(seed)
    M = N * HW * HW
    h2 = torch.randn(N, HW, HW, C, device=DEV, generator=g).bfloat16()
    scale = 0.1 * (0.5 + torch.rand(C, device=DEV, generator=g))
    shift = shift_level * (0.75 + 0.5 * torch.rand(C, device=DEV, generator=g))
    # BN2 coefficients as bn_coef lays them out: [scale, shift, mean, invstd] (h2 ~ N(0, 1): mean 0, invstd 1)
    c2 = torch.stack([scale, shift, torch.zeros(C, device=DEV), torch.ones(C, device=DEV)]).float().contiguous()
    # every output row one sign: h3 = a2 W^T has a large common-mode part in every channel
    sign = torch.where(torch.rand(Cout, 1, device=DEV, generator=g) < 0.5, -1.0, 1.0)
    w = (sign * torch.rand(Cout, C, device=DEV, generator=g).add_(0.05) * C ** -0.5).bfloat16()
    return M, h2, c2, w.reshape(Cout, 1, 1, C).contiguous()


@pytest.mark.parametrize("shift_level", [3.0, 12.0])
def test_gram_bn3_large_mean_per_channel(shift_level):
    X = ext()
    C, Cout, N, HW = 64, 256, 512, 56
    M, h2, c2, w = _case(C, Cout, N, HW, 7, shift_level)
    assert M >= 1_600_000
    eps = 1e-5
    gamma = torch.ones(Cout, device=DEV)
    beta = torch.zeros(Cout, device=DEV)
    G, s = X.bn_gram(h2, c2)
    coef3, u = X.bn_gram_coef(G, s, w, M, gamma, beta, None, None, 0.1, eps)

    # fp64 reference over the exact bf16 operand conv3 multiplies, in row chunks
    W = w.reshape(Cout, C).double()
    sum_h = torch.zeros(Cout, dtype=torch.float64, device=DEV)
    chunk = 1 << 18
    a_rows = h2.reshape(M, C)

    def a_of(r0):
        return torch.relu(a_rows[r0:r0 + chunk].float() * c2[0] + c2[1]).bfloat16().double()

    for r0 in range(0, M, chunk):
        sum_h += (a_of(r0) @ W.t()).sum(0)
    mean = sum_h / M
    ssd = torch.zeros(Cout, dtype=torch.float64, device=DEV)
    for r0 in range(0, M, chunk):
        ssd += ((a_of(r0) @ W.t() - mean) ** 2).sum(0)
    var = ssd / M
    ratio = (mean.abs() / var.sqrt()).min().item()
    assert ratio >= 30, f"test setup: min |mean|/std {ratio:.1f}"

    var_ours = 1.0 / coef3[3].double() ** 2 - eps
    mean_ours = coef3[2].double()
    ev = ((var_ours - var).abs() / var).max().item()
    em = ((mean_ours - mean).abs() / mean.abs()).max().item()
    print(f"\nshift {shift_level}: min |mean|/std {ratio:.0f}; per-channel rel err var {ev:.2e} mean {em:.2e}")
    assert ev < 1e-3, f"BN3 variance per-channel rel err {ev:.3e}"
    assert em < 1e-4, f"BN3 mean per-channel rel err {em:.3e}"

    # backward: dz3 random, P = dz3^T a2 by the same weight-grad GEMM the model runs
    gz = torch.Generator(device=DEV).manual_seed(11)
    dz = torch.randn(N, HW, HW, Cout, device=DEV, generator=gz).bfloat16()
    P = torch.zeros(Cout, 1, 1, C, dtype=torch.float32, device=DEV)
    X.conv_wgrad(dz, h2, P, [1, 1], [0, 0], [1, 1], 1.0, c2, deterministic=True)
    dzr = dz.reshape(M, Cout)
    part = torch.zeros(2, Cout, 1, device=DEV)
    part[0, :, 0] = dzr.float().sum(0)
    dg, db = torch.zeros(Cout, device=DEV), torch.zeros(Cout, device=DEV)
    dw = torch.zeros(Cout, 1, 1, C, device=DEV)
    X.bn_gram_bwd(part, P.reshape(Cout, C).contiguous(), w, u, s, coef3, gamma, M, dg, db, dw)

    # fp64: Sdzx = sum dz (h - mean) / std; dW3 = sum_r dh[r] a2[r] with dh = a dz + b h + c
    invstd = 1.0 / torch.sqrt(var + eps)
    sdz = torch.zeros(Cout, dtype=torch.float64, device=DEV)
    sdzx = torch.zeros(Cout, dtype=torch.float64, device=DEV)
    sq = torch.zeros(Cout, dtype=torch.float64, device=DEV)
    for r0 in range(0, M, chunk):
        d = dzr[r0:r0 + chunk].double()
        sdz += d.sum(0)
        t = d * (a_of(r0) @ W.t() - mean)
        sdzx += t.sum(0)
        sq += (t * t).sum(0)
    sdzx *= invstd
    # a random-sign sum can land near 0 in some channel: its error is measured against the larger of its
    # value and its natural magnitude sqrt(sum of squared terms) (both per channel)
    scale = torch.maximum(sdzx.abs(), invstd * sq.sqrt())
    A = invstd  # gamma = 1
    B = -A * invstd * sdzx / M
    Cc = -A * sdz / M - B * mean
    dW = torch.zeros(Cout, C, dtype=torch.float64, device=DEV)
    for r0 in range(0, M, chunk):
        a = a_of(r0)
        dh = dzr[r0:r0 + chunk].double() * A + (a @ W.t()) * B + Cc
        dW += dh.t() @ a
    eg = ((dg.double() - sdzx).abs() / scale).max().item()
    ew = ((dw.reshape(Cout, C).double() - dW).norm(dim=1) / dW.norm(dim=1)).max().item()
    print(f"per-channel rel err dgamma {eg:.2e}, dW3 rows {ew:.2e}")
    assert eg < 1e-3, f"BN3 dgamma (Sdzx) per-channel rel err {eg:.3e}"
    assert ew < 1e-3, f"dW3 per-row rel err {ew:.3e}"
