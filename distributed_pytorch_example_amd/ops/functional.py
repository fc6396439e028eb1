"""Autograd-level ops.  GPU tensors -> hand-written gfx950 kernels (``_C``);
CPU tensors -> torch reference math with identical semantics (the CPU/gloo
configuration of the reference, and the reference used by the numerics tests).

Activation layout convention: convolutional activations are NHWC
(``[N, H, W, C]``); on the GPU they are bf16.  Conv weights are stored
``[Cout, R, S, Cin]`` (OHWI) so the forward implicit GEMM reads them K-contiguous.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import torch
import torch.nn.functional as F
from torch.autograd import Function

from ._ext import ext
from ._state import grad_done, grad_fresh, grad_sink, note_use, shadow

ACT_NONE, ACT_RELU, ACT_GELU = 0, 1, 2

# CPU reference path: optionally round activations (forward) and their
# gradients (backward) to bf16 at the same points the GPU kernels do, so the
# GPU path can be validated against a reference with identical rounding
# points (tests) instead of against pure fp32.
EMULATE_BF16 = False


class _RoundBF16(Function):
    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


def _emu(x):
    return _RoundBF16.apply(x) if EMULATE_BF16 else x


def _emu_w(w):
    return w.to(torch.bfloat16).to(w.dtype) if EMULATE_BF16 else w


def _pad8(n: int) -> int:
    return (n + 7) // 8 * 8


# ===================================================================== Linear
class _LinearFn(Function):
    """bf16 Linear on the MFMA GEMMs.  Output widths that are not a multiple of 8 (SimpleNet's
    10-class head) run on the bf16 shadow padded to Np = pad8(N) rows: bias (zero-padded) and ReLU
    stay in the GEMM epilogue, the backward pads dy once (F.pad, one kernel) and the weight grad
    writes only the N real rows into the gradient buffer, with the bias grad from the same launch."""

    @staticmethod
    def forward(ctx, x, weight, bias, act: int, out_f32: bool):
        C = ext()
        N = weight.shape[0]
        Np = _pad8(N)
        w16 = shadow(weight, Np - N)
        xb = x if x.dtype == torch.bfloat16 else x.to(torch.bfloat16)
        xb = xb.contiguous()
        if Np != N:
            bpad = F.pad(bias.detach(), (0, Np - N)) if bias is not None else None
            y = C.linear_fwd(xb, w16, bpad, act, out_f32)[..., :N].contiguous()
        else:
            y = C.linear_fwd(xb, w16, bias.detach() if bias is not None else None, act, out_f32)
        ctx.save_for_backward(xb, y if act != ACT_NONE else None)
        ctx.weight, ctx.bias, ctx.act, ctx.N, ctx.Np = weight, bias, act, N, Np
        ctx.x_dtype = x.dtype
        note_use(weight)
        if bias is not None:
            note_use(bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = ext()
        xb, y = ctx.saved_tensors
        weight, bias, act, N, Np = ctx.weight, ctx.bias, ctx.act, ctx.N, ctx.Np
        dy = dy.to(torch.bfloat16) if dy.dtype != torch.bfloat16 else dy
        if act == ACT_RELU:
            dy = C.act(dy.contiguous(), y.to(torch.bfloat16).contiguous() if y.dtype != torch.bfloat16 else y.contiguous(), 1)
        dy = dy.contiguous()
        dyp = F.pad(dy, (0, Np - N)) if Np != N else dy  # zero pad columns: the GEMMs' 16-B rows
        dx = None
        if ctx.needs_input_grad[0]:
            dx = C.linear_dgrad(dyp, shadow(weight, Np - N))
            if ctx.x_dtype != torch.bfloat16:
                dx = dx.to(ctx.x_dtype)
        want_b = bias is not None and ctx.needs_input_grad[2]
        bbuf, bdirect = grad_sink(bias) if want_b else (None, False)
        gw = None
        if ctx.needs_input_grad[1]:
            buf, direct = grad_sink(weight)
            # column-padded dy: only the N real rows of dW (and of db) are written
            C.linear_wgrad(dyp, xb, buf, 1.0, None, bbuf, 0, direct and grad_fresh(weight))
            grad_done(weight, direct)
            gw = None if direct else buf
        elif want_b:
            C.colsum(dy, bbuf, True)
        gb = None
        if want_b:
            grad_done(bias, bdirect)
            gb = None if bdirect else bbuf
        return dx, gw, gb, None, None


def linear(x, weight, bias=None, act: int = ACT_NONE, out_f32: bool = False):
    if not x.is_cuda:
        xin = _emu(x.float() if x.dtype != weight.dtype else x)
        w = weight + (_emu_w(weight) - weight).detach() if EMULATE_BF16 else weight
        y = F.linear(xin, w, bias)
        if act == ACT_RELU:
            y = F.relu(y)
        elif act == ACT_GELU:
            y = F.gelu(y, approximate="tanh")
        return y if out_f32 else _emu(y)
    if act == ACT_GELU:
        return gelu(_LinearFn.apply(x, weight, bias, ACT_NONE, out_f32))
    return _LinearFn.apply(x, weight, bias, act, out_f32)


# ============================================================ activations
class _ActFn(Function):
    @staticmethod
    def forward(ctx, x, op: int):
        C = ext()
        xc = x.contiguous()
        y = C.act(xc, None, op)
        ctx.op = op
        ctx.save_for_backward(y if op == 0 else xc)
        return y

    @staticmethod
    def backward(ctx, dy):
        (s,) = ctx.saved_tensors
        dy = dy.contiguous().to(s.dtype)
        return ext().act(dy, s, 1 if ctx.op == 0 else 3), None


def relu(x):
    if not x.is_cuda:
        return F.relu(x)
    return _ActFn.apply(x, 0)


def gelu(x):
    if not x.is_cuda:
        return F.gelu(x, approximate="tanh")
    return _ActFn.apply(x, 2)


class _RNG:
    """Counter-based dropout RNG stream: (seed, offset) -> Philox; mask regenerated in backward."""

    seed = None
    offset = 0

    @classmethod
    def next(cls, n: int):
        if cls.seed is None:
            cls.seed = int(torch.initial_seed()) & 0xFFFFFFFFFFFF
        off = cls.offset
        cls.offset += (n + 3) // 4
        return cls.seed, off


class _DropoutFn(Function):
    @staticmethod
    def forward(ctx, x, p: float):
        seed, off = _RNG.next(x.numel())
        ctx.p, ctx.seed, ctx.off = p, seed, off
        return ext().dropout(x.contiguous(), p, seed, off)

    @staticmethod
    def backward(ctx, dy):
        return ext().dropout(dy.contiguous(), ctx.p, ctx.seed, ctx.off), None


def dropout(x, p: float, training: bool):
    if not training or p == 0.0:
        return x
    if not x.is_cuda:
        return F.dropout(x, p, True)
    return _DropoutFn.apply(x, p)


# ====================================================================== Conv
def _conv_out(h, k, s, p, d):
    return (h + 2 * p - d * (k - 1) - 1) // s + 1


class _ConvFn(Function):
    @staticmethod
    def forward(ctx, x, weight, w16, stride, padding, dilation, want_stats):
        C = ext()
        y, st = C.conv_fwd(x, w16, list(stride), list(padding), list(dilation), want_stats, None)
        ctx.save_for_backward(x)
        ctx.w16, ctx.weight = w16, weight
        ctx.conf = (list(stride), list(padding), list(dilation))
        note_use(weight)
        if want_stats:
            ctx.mark_non_differentiable(st)
            return y, st
        return y

    @staticmethod
    def backward(ctx, dy, *unused):
        C = ext()
        (x,) = ctx.saved_tensors
        stride, padding, dilation = ctx.conf
        dy = dy.contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            dx = C.conv_dgrad(dy, ctx.w16, list(x.shape), stride, padding, dilation, None)
        gw = None
        weight = ctx.weight
        if ctx.needs_input_grad[1]:
            if tuple(ctx.w16.shape) == tuple(weight.shape):
                buf, direct = grad_sink(weight)
                C.conv_wgrad(dy, x, buf, stride, padding, dilation, 1.0)
            else:  # channel-padded filter (stem): reduce in padded layout, keep the real channels
                tmp = torch.zeros(ctx.w16.shape, dtype=torch.float32, device=dy.device)
                C.conv_wgrad(dy, x, tmp, stride, padding, dilation, 1.0)
                buf, direct = grad_sink(weight)
                buf.add_(tmp[..., : weight.shape[-1]])
            grad_done(weight, direct)
            gw = None if direct else buf
        return dx, gw, None, None, None, None, None


def _pad_filter_channels(cp: int):
    def fn(w):
        out = torch.zeros((*w.shape[:-1], cp), dtype=torch.bfloat16, device=w.device)
        out[..., : w.shape[-1]] = w
        return out

    return fn


def conv2d_nhwc(x, weight, stride=(1, 1), padding=(0, 0), dilation=(1, 1), want_stats: bool = False):
    """x: [N,H,W,Cin'] (Cin' >= Cin, zero-padded channels allowed), weight: [Cout,R,S,Cin] fp32 master.

    With ``want_stats`` (GPU) returns ``(y, stats)`` where ``stats`` holds per-channel
    partial (sum, sum^2) of y from the GEMM epilogue, consumed by ``batch_norm_nhwc``."""
    stride, padding, dilation = _pair(stride), _pair(padding), _pair(dilation)
    if not x.is_cuda:
        cin = weight.shape[-1]
        xc = _emu(x[..., :cin].permute(0, 3, 1, 2).float())
        w = weight + (_emu_w(weight) - weight).detach() if EMULATE_BF16 else weight
        y = F.conv2d(xc, w.permute(0, 3, 1, 2), None, stride, padding, dilation)
        y = _emu(y.permute(0, 2, 3, 1).contiguous())
        return (y, None) if want_stats else y
    from ._state import derived_shadow

    if x.shape[-1] != weight.shape[-1]:
        w16 = derived_shadow(weight, f"cpad{x.shape[-1]}", _pad_filter_channels(x.shape[-1]))
    else:
        w16 = shadow(weight)
    return _ConvFn.apply(x.contiguous(), weight, w16, stride, padding, dilation, want_stats)


# ================================================ space-to-depth ResNet stem
# A 7x7/s2/p3 conv over x equals a 4x4/s1 conv over the space-to-depth image
# x'[q][p][(ay,ax,c)] = x[2q+ay][2p+ax][c], padded 2 (top/left) and 1
# (bottom/right), with filter w'[o][dy][dx][(ay,ax,c)] = w[o][2dy+ay-1][2dx+ax-1][c]
# (zero outside 7x7).  Each 7x7 tap appears exactly once in w', so the weight
# gradient maps back by a gather.
_S2D_IDX: dict = {}


def _s2d_index(cin: int, device):
    key = (cin, str(device))
    if key not in _S2D_IDX:
        dst, src = [], []
        for dy in range(4):
            for dx in range(4):
                for ay in range(2):
                    for ax in range(2):
                        for c in range(4):
                            r, s_ = 2 * dy + ay - 1, 2 * dx + ax - 1
                            if 0 <= r < 7 and 0 <= s_ < 7 and c < cin:
                                dst.append(((dy * 4 + dx) * 4 + ay * 2 + ax) * 4 + c)
                                src.append((r * 7 + s_) * cin + c)
        order = sorted(range(len(src)), key=lambda i: src[i])
        inv = torch.tensor([dst[i] for i in order], dtype=torch.long, device=device)  # w-flat index -> w'-flat index
        _S2D_IDX[key] = (torch.tensor(dst, dtype=torch.long, device=device),
                         torch.tensor(src, dtype=torch.long, device=device), inv)
    return _S2D_IDX[key]


def _s2d_filter(w):
    co, cin = w.shape[0], w.shape[-1]
    dst, src, _ = _s2d_index(cin, w.device)
    out = torch.zeros((co, 256), dtype=torch.bfloat16, device=w.device)
    out[:, dst] = w.reshape(co, -1)[:, src].to(torch.bfloat16)
    return out.view(co, 4, 4, 16)


class _S2DStemFn(Function):
    @staticmethod
    def forward(ctx, xs, weight, w16, want_stats):
        y, st = ext().conv_fwd(xs, w16, [1, 1], [2, 2, 1, 1], [1, 1], want_stats, None)
        ctx.save_for_backward(xs)
        ctx.weight = weight
        note_use(weight)
        if want_stats:
            ctx.mark_non_differentiable(st)
            return y, st
        return y

    @staticmethod
    def backward(ctx, dy, *unused):
        (xs,) = ctx.saved_tensors
        weight = ctx.weight
        co = weight.shape[0]
        tmp = torch.zeros((co, 4, 4, 16), dtype=torch.float32, device=dy.device)
        ext().conv_wgrad(dy.contiguous(), xs, tmp, [1, 1], [2, 2], [1, 1], 1.0)
        buf, direct = grad_sink(weight)
        buf.view(co, -1).add_(tmp.view(co, 256)[:, _s2d_index(weight.shape[-1], dy.device)[2]])
        grad_done(weight, direct)
        return None, (None if direct else buf), None, None


def to_s2d_input(x: torch.Tensor) -> torch.Tensor:
    """NCHW fp32 images [N,3,H,W] -> space-to-depth NHWC bf16 [N,H/2,W/2,16] (GPU stem input)."""
    return ext().nchw_to_s2d(x.float().contiguous())


def stem_conv_s2d(xs, weight, want_stats: bool = False):
    """7x7/s2/p3 conv (filter ``weight`` [Co,7,7,Cin<=4]) over a space-to-depth input ``xs``."""
    from ._state import derived_shadow

    assert tuple(weight.shape[1:3]) == (7, 7) and weight.shape[-1] <= 4 and xs.shape[-1] == 16
    w16 = derived_shadow(weight, "s2d", _s2d_filter)
    return _S2DStemFn.apply(xs.contiguous(), weight, w16, want_stats)


def _pair(v) -> tuple:
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


# ================================================================ BatchNorm
class _BNFn(Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, residual, rmean, rvar, momentum, eps, relu_, stats):
        C = ext()
        y, coef = C.bn_fwd_train(x, gamma.detach(), beta.detach(), rmean, rvar, momentum, eps, relu_, residual, stats)
        ctx.save_for_backward(x, y if relu_ else None, coef)
        ctx.gamma, ctx.beta, ctx.has_res = gamma, beta, residual is not None
        note_use(gamma)
        note_use(beta)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = ext()
        x, y, coef = ctx.saved_tensors
        gbuf, gdirect = grad_sink(ctx.gamma)
        bbuf, bdirect = grad_sink(ctx.beta)
        dx, dz = C.bn_bwd(dy.contiguous(), y, x, ctx.gamma.detach(), coef, gbuf, bbuf, ctx.has_res)
        grad_done(ctx.gamma, gdirect)
        grad_done(ctx.beta, bdirect)
        return (dx, None if gdirect else gbuf, None if bdirect else bbuf, dz if ctx.has_res else None,
                None, None, None, None, None, None)


def batch_norm_nhwc(x, gamma, beta, running_mean, running_var, training: bool, momentum: float = 0.1,
                    eps: float = 1e-5, relu: bool = False, residual=None, stats=None, num_batches_tracked=None):
    """y = act(BN(x) [+ residual]) over the channel (last) dim of an NHWC tensor."""
    if not x.is_cuda:
        C_ = x.shape[-1]
        xf = x.reshape(-1, C_).float()
        yf = F.batch_norm(xf, running_mean, running_var, gamma, beta, training, momentum, eps)
        y = yf.reshape(x.shape)
        if residual is not None:
            y = y + residual.float()
        if relu:
            y = F.relu(y)
        if training and num_batches_tracked is not None:
            num_batches_tracked.add_(1)
        return _emu(y)
    if training:
        if num_batches_tracked is not None:
            num_batches_tracked.add_(1)
        return _BNFn.apply(x.contiguous(), gamma, beta, residual.contiguous() if residual is not None else None,
                           running_mean, running_var, momentum, eps, relu, stats)
    return ext().bn_fwd_eval(x.contiguous(), gamma.detach(), beta.detach(), running_mean, running_var, eps, relu,
                             residual.contiguous() if residual is not None else None)


class _StemBNReluPoolFn(Function):
    """maxpool(relu(BN(h))) for the ResNet stem with training-mode BN whose
    statistics came from the conv epilogue: the BN+ReLU output (the largest
    activation of the network) is never written or re-read; the backward
    gathers the pooled gradient per element inside the BN-backward passes."""

    @staticmethod
    def forward(ctx, h, gamma, beta, rmean, rvar, momentum, eps, stats, k, s, p):
        C = ext()
        M = h.numel() // h.shape[-1]
        coef = C.bn_coef(stats, M, gamma.detach(), beta.detach(), rmean, rvar, momentum, eps)
        y, idx = C.bnrelu_maxpool_fwd(h, coef, k, s, p)
        ctx.save_for_backward(h, idx, coef)
        ctx.gamma, ctx.beta, ctx.conf = gamma, beta, (k, s, p)
        note_use(gamma)
        note_use(beta)
        return y

    @staticmethod
    def backward(ctx, dy):
        h, idx, coef = ctx.saved_tensors
        gbuf, gdirect = grad_sink(ctx.gamma)
        bbuf, bdirect = grad_sink(ctx.beta)
        dh = ext().maxpool_bn_bwd(dy.contiguous(), idx, h, ctx.gamma.detach(), coef, gbuf, bbuf, *ctx.conf)
        grad_done(ctx.gamma, gdirect)
        grad_done(ctx.beta, bdirect)
        return (dh, None if gdirect else gbuf, None if bdirect else bbuf) + (None,) * 8


def stem_bn_relu_maxpool(h, bn, stats, kernel_size=3, stride=2, padding=1):
    """max_pool2d(relu(bn(h))) in training mode from conv-epilogue statistics (GPU)."""
    if bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
    return _StemBNReluPoolFn.apply(h.contiguous(), bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.momentum, bn.eps,
                                   stats, kernel_size, stride, padding)


class _StemFusedFn(Function):
    """The whole training-mode ResNet stem -- s2d 7x7/s2 conv, BN (statistics from the conv epilogue), ReLU,
    3x3/s2 max-pool -- as one node.  Backward: the BN-backward reduction over the pooled gradient, then the
    stem weight grad computing dL/dh on the fly (csrc stem_bwd_fused): neither the BN+ReLU output nor dL/dh
    is ever written (the standalone apply pass moved 1.95 GB per batch-512 step)."""

    @staticmethod
    def forward(ctx, xs, weight, w16, gamma, beta, rmean, rvar, momentum, eps):
        C = ext()
        h, st = C.conv_fwd(xs, w16, [1, 1], [2, 2, 1, 1], [1, 1], True, None)
        coef = C.bn_coef(st, h.numel() // h.shape[-1], gamma.detach(), beta.detach(), rmean, rvar, momentum, eps)
        y, idx = C.bnrelu_maxpool_fwd(h, coef, 3, 2, 1)
        ctx.save_for_backward(xs, h, idx, coef)
        ctx.weight, ctx.gamma, ctx.beta = weight, gamma, beta
        for p in (weight, gamma, beta):
            note_use(p)
        return y

    @staticmethod
    def backward(ctx, dy):
        xs, h, idx, coef = ctx.saved_tensors
        weight, gamma, beta = ctx.weight, ctx.gamma, ctx.beta
        co = weight.shape[0]
        gbuf, gdirect = grad_sink(gamma)
        bbuf, bdirect = grad_sink(beta)
        tmp = torch.zeros((co, 4, 4, 16), dtype=torch.float32, device=dy.device)
        ext().stem_bwd_fused(dy.contiguous(), idx, h, xs, gamma.detach(), coef, gbuf, bbuf, tmp)
        grad_done(gamma, gdirect)
        grad_done(beta, bdirect)
        buf, direct = grad_sink(weight)
        buf.view(co, -1).add_(tmp.view(co, 256)[:, _s2d_index(weight.shape[-1], dy.device)[2]])
        grad_done(weight, direct)
        return (None, None if direct else buf, None, None if gdirect else gbuf, None if bdirect else bbuf,
                None, None, None, None)


def stem_fused_ok(xs) -> bool:
    """The fused stem path's envelope: s2d input [N, H, W, 16] on the GPU with even H, W <= 112."""
    return (xs.is_cuda and xs.dim() == 4 and xs.shape[-1] == 16 and xs.shape[1] % 2 == 0 and xs.shape[2] % 2 == 0
            and 97 <= xs.shape[2] <= 112 and xs.shape[1] >= 8)


def stem_fused(xs, weight, bn):
    """maxpool(relu(bn(conv_s2d(xs, weight)))) in training mode, one autograd node (see _StemFusedFn)."""
    from ._state import derived_shadow

    if bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
    w16 = derived_shadow(weight, "s2d", _s2d_filter)
    return _StemFusedFn.apply(xs.contiguous(), weight, w16, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                              bn.momentum, bn.eps)


# ================================================================== pooling
class _MaxPoolFn(Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        y, idx = ext().maxpool_fwd(x, k, s, p)
        ctx.save_for_backward(idx)
        ctx.conf = (list(x.shape), k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        xs, k, s, p = ctx.conf
        return ext().maxpool_bwd(dy.contiguous(), idx, xs, k, s, p), None, None, None


def max_pool2d_nhwc(x, kernel_size=3, stride=2, padding=1):
    if not x.is_cuda:
        return _emu(F.max_pool2d(x.permute(0, 3, 1, 2), kernel_size, stride, padding).permute(0, 2, 3, 1).contiguous())
    return _MaxPoolFn.apply(x.contiguous(), kernel_size, stride, padding)


class _GAvgPoolFn(Function):
    @staticmethod
    def forward(ctx, x):
        ctx.shape = list(x.shape)
        return ext().gavgpool_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        return ext().gavgpool_bwd(dy.contiguous(), ctx.shape)


def global_avg_pool_nhwc(x):
    if not x.is_cuda:
        return _emu(x.float().mean(dim=(1, 2)))
    return _GAvgPoolFn.apply(x.contiguous())


# ===================================================================== loss
class _CEFn(Function):
    """Mean CE: the kernel pair (per-row pass + fixed-order reduction) also yields the mean over the
    non-ignored rows and 1 / their count, and backward is one scaling pass -- no torch-level count /
    clamp / divide / cast kernels at the launch-bound forward -> backward seam."""

    @staticmethod
    def forward(ctx, logits, labels, num_classes: int, ignore_index: int):
        out4, d = ext().cross_entropy_mean(logits.contiguous(), labels.contiguous(), num_classes,
                                           logits.dtype == torch.bfloat16, ignore_index)
        ctx.save_for_backward(d, out4)
        return out4[2:3].reshape(())

    @staticmethod
    def backward(ctx, g):
        d, out4 = ctx.saved_tensors
        return ext().ce_grad_scale(d, g.float().reshape(1), out4[3:4]), None, None, None


def cross_entropy(logits, labels, num_classes: Optional[int] = None, ignore_index: int = -100):
    """Mean softmax cross-entropy over rows (torch.nn.CrossEntropyLoss semantics)."""
    if num_classes is None:
        num_classes = logits.shape[-1]
    if not logits.is_cuda:
        return F.cross_entropy(logits.reshape(-1, logits.shape[-1])[:, :num_classes].float(), labels.reshape(-1),
                               ignore_index=ignore_index)
    return _CEFn.apply(logits.reshape(-1, logits.shape[-1]), labels.reshape(-1), num_classes, ignore_index)


def cross_entropy_eval(logits, labels, num_classes: Optional[int] = None):
    """(loss_sum, correct_count) as device scalars, one fused pass (no grad)."""
    if num_classes is None:
        num_classes = logits.shape[-1]
    if not logits.is_cuda:
        lf = logits.reshape(-1, logits.shape[-1])[:, :num_classes].float()
        loss = F.cross_entropy(lf, labels.reshape(-1), reduction="sum")
        return loss, (lf.argmax(1) == labels.reshape(-1)).sum().float()
    _, s, correct, _ = ext().cross_entropy(logits.reshape(-1, logits.shape[-1]).contiguous(), labels.reshape(-1).contiguous(),
                                           num_classes, 1.0, False, False, -100)
    return s.reshape(()), correct.reshape(())


# ================================================================ LayerNorm
class _LNFn(Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        y, mean, rstd = ext().layernorm_fwd(x.contiguous(), w.detach(), b.detach() if b is not None else None, eps)
        ctx.save_for_backward(x, mean, rstd)
        ctx.w, ctx.b = w, b
        note_use(w)
        if b is not None:
            note_use(b)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, rstd = ctx.saved_tensors
        wbuf, wd = grad_sink(ctx.w)
        bbuf, bd = (grad_sink(ctx.b) if ctx.b is not None else (None, False))
        dx = ext().layernorm_bwd(dy.contiguous().to(torch.bfloat16), x.contiguous(), ctx.w.detach(), mean, rstd, wbuf, bbuf,
                                 None)
        grad_done(ctx.w, wd)
        if ctx.b is not None:
            grad_done(ctx.b, bd)
        return dx, (None if wd else wbuf), (None if (bd or ctx.b is None) else bbuf), None


def layer_norm(x, weight, bias=None, eps: float = 1e-5):
    """LayerNorm over the last dim. GPU: f32/bf16 in -> bf16 out."""
    if not x.is_cuda:
        return F.layer_norm(x.float(), (x.shape[-1],), weight, bias, eps)
    return _LNFn.apply(x, weight, bias, eps)


# ================================================================ Embedding
class _EmbFn(Function):
    @staticmethod
    def forward(ctx, idx, wte, wpe, wte16, wpe16):
        out = ext().embedding_fwd(idx, wte16, wpe16)
        ctx.save_for_backward(idx)
        ctx.wte, ctx.wpe = wte, wpe
        note_use(wte)
        if wpe is not None:
            note_use(wpe)
        return out

    @staticmethod
    def backward(ctx, dout):
        (idx,) = ctx.saved_tensors
        tb, td = grad_sink(ctx.wte)
        pb, pd = grad_sink(ctx.wpe) if ctx.wpe is not None else (None, False)
        for p, buf, d in ((ctx.wte, tb, td), (ctx.wpe, pb, pd)):  # the scatter-add needs a zeroed start
            if p is not None and d and grad_fresh(p):
                buf.zero_()
        ext().embedding_bwd(idx, dout.contiguous().float(), tb, pb)
        grad_done(ctx.wte, td)
        if ctx.wpe is not None:
            grad_done(ctx.wpe, pd)
        return None, (None if td else tb), (None if (pd or ctx.wpe is None) else pb), None, None


def embedding(idx, wte, wpe=None):
    """tok + pos embedding -> f32 [B,T,D] residual stream."""
    if not idx.is_cuda:
        T = idx.shape[1]
        x = F.embedding(idx, wte)
        if wpe is not None:
            x = x + wpe[:T].unsqueeze(0)
        return x
    return _EmbFn.apply(idx, wte, wpe, shadow(wte), shadow(wpe) if wpe is not None else None)


# ================================================================ Attention
class _AttnFn(Function):
    @staticmethod
    def forward(ctx, qkv, H: int, scale: float):
        out, lse = ext().attn_fwd(qkv.contiguous(), H, scale, True)
        ctx.save_for_backward(qkv, out, lse)
        ctx.H, ctx.scale = H, scale
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        dqkv = ext().attn_bwd(qkv, out, dout.contiguous().to(torch.bfloat16), lse, ctx.H, ctx.scale, True)
        return dqkv, None, None


def causal_attention(qkv, n_head: int):
    """qkv: [B, T, 3*H*D] -> [B, T, H*D] causal softmax attention."""
    B, T, three_hd = qkv.shape
    D = three_hd // (3 * n_head)
    scale = 1.0 / math.sqrt(D)
    if not qkv.is_cuda:
        q, k, v = qkv.float().view(B, T, 3, n_head, D).permute(2, 0, 3, 1, 4)
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        return o.transpose(1, 2).reshape(B, T, n_head * D)
    out = _AttnFn.apply(qkv.reshape(B, T, 3, n_head, D), n_head, scale)
    return out.reshape(B, T, n_head * D)


def add(a, b):
    if not a.is_cuda:
        return a + b
    return _AddFn.apply(a, b)


class _AddFn(Function):
    @staticmethod
    def forward(ctx, a, b):
        return ext().add(a.contiguous(), b.contiguous(), 1.0)

    @staticmethod
    def backward(ctx, g):
        return g, g


def to_nhwc_input(x: torch.Tensor, cpad: int = 8) -> torch.Tensor:
    """NCHW fp32 image batch -> NHWC (bf16 on GPU, channel-padded to ``cpad``)."""
    if not x.is_cuda:
        y = x.permute(0, 2, 3, 1).float()
        if y.shape[-1] < cpad:
            y = F.pad(y, (0, cpad - y.shape[-1]))
        return y.contiguous()
    return ext().nchw_to_nhwc(x.float().contiguous(), cpad)


# ====================================================== residual-stream linear
class _LinearResidualFn(Function):
    """y = x_res + a @ W^T + b  with a bf16 activations and x_res the fp32 residual stream,
    one GEMM launch (fp32-residual epilogue)."""

    @staticmethod
    def forward(ctx, a, weight, bias, x_res):
        C = ext()
        w16 = shadow(weight)
        ab = a.contiguous() if a.dtype == torch.bfloat16 else a.to(torch.bfloat16).contiguous()
        y = C.linear_fwd(ab, w16, bias.detach() if bias is not None else None, 0, True, x_res.contiguous(), None)
        ctx.save_for_backward(ab)
        ctx.weight, ctx.bias = weight, bias
        note_use(weight)
        if bias is not None:
            note_use(bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = ext()
        (ab,) = ctx.saved_tensors
        weight, bias = ctx.weight, ctx.bias
        dyb = dy.to(torch.bfloat16).contiguous()
        da = C.linear_dgrad(dyb, shadow(weight)) if ctx.needs_input_grad[0] else None
        buf, direct = grad_sink(weight)
        bb, bd = grad_sink(bias) if bias is not None else (None, False)
        C.linear_wgrad(dyb, ab, buf, 1.0, None, bb, 0, direct and grad_fresh(weight))  # bias grad: row sums of dy^T in the same launch
        grad_done(weight, direct)
        gb = None
        if bias is not None:
            grad_done(bias, bd)
            gb = None if bd else bb
        return da, (None if direct else buf), gb, dy


def linear_residual(a, weight, bias, x_res):
    """x_res (fp32) + linear(a)."""
    if not a.is_cuda:
        return x_res + F.linear(a.float(), weight, bias)
    return _LinearResidualFn.apply(a, weight, bias, x_res)


# ================================================================ LM head
class _LMHeadFn(Function):
    """logits[.., Vp] = x @ wte_pad^T, wte tied with the token embedding; the
    vocab is padded to a multiple of 64 inside the bf16 shadow only (zero pad
    rows), the fp32 master keeps the canonical [V, D] shape."""

    @staticmethod
    def forward(ctx, x, wte, pad_rows: int):
        C = ext()
        w16 = shadow(wte, pad_rows)
        xb = x.contiguous() if x.dtype == torch.bfloat16 else x.to(torch.bfloat16).contiguous()
        y = C.linear_fwd(xb, w16, None, 0, False, None, None)
        ctx.save_for_backward(xb)
        ctx.wte, ctx.pad = wte, pad_rows
        note_use(wte)
        return y

    @staticmethod
    def backward(ctx, dlogits):
        C = ext()
        (xb,) = ctx.saved_tensors
        d = dlogits.to(torch.bfloat16).contiguous()
        dx = C.linear_dgrad(d, shadow(ctx.wte, ctx.pad))
        buf, direct = grad_sink(ctx.wte)
        C.linear_wgrad(d, xb, buf, 1.0, None, None, 0, direct and grad_fresh(ctx.wte))  # padded leading dim, only the V real rows are produced
        grad_done(ctx.wte, direct)
        return dx, (None if direct else buf), None


class _LMHeadCEFn(Function):
    """Fused tied LM head + mean cross-entropy (GPT-2 training path).

    The logits never leave the op: the CE kernel holds each row in registers
    and overwrites the logits with (softmax - onehot) in place (one HBM read +
    one write of the [tokens, Vp] matrix); backward feeds that straight to the
    dgrad/wgrad GEMMs, which read the incoming loss gradient / N as a device
    scalar (``alpha_t``) -- no separate scaling pass over the 0.8 GB gradient.
    """

    @staticmethod
    def forward(ctx, x, wte, labels, pad_rows: int, ignore_index: int):
        C = ext()
        w16 = shadow(wte, pad_rows)
        xb = x.contiguous() if x.dtype == torch.bfloat16 else x.to(torch.bfloat16).contiguous()
        xb = xb.reshape(-1, xb.shape[-1])
        logits = C.linear_fwd(xb, w16, None, 0, False, None, None)
        lab = labels.reshape(-1).contiguous()
        out4, d = C.cross_entropy_mean(logits, lab, wte.shape[0], True, ignore_index, True)
        ctx.save_for_backward(xb, d, out4)
        ctx.wte, ctx.pad, ctx.xshape = wte, pad_rows, x.shape
        note_use(wte)
        return out4[2:3].reshape(())  # mean over the non-ignored tokens (kernel-side count)

    @staticmethod
    def backward(ctx, g):
        C = ext()
        xb, d, out4 = ctx.saved_tensors
        scale = g.float().reshape(1) * out4[3:4]  # dL/dlogits = (softmax - onehot) * g / n, applied by the GEMMs
        dx = C.linear_dgrad(d, shadow(ctx.wte, ctx.pad), None, scale)
        buf, direct = grad_sink(ctx.wte)
        C.linear_wgrad(d, xb, buf, 1.0, scale, None, 0, direct and grad_fresh(ctx.wte))
        grad_done(ctx.wte, direct)
        return dx.reshape(ctx.xshape), (None if direct else buf), None, None, None


def lm_head_ce(x, wte, labels, vocab_pad_to: int = 64, ignore_index: int = -100):
    """Mean CE of the tied LM head logits ``x @ wte^T`` against ``labels`` (fused)."""
    if not x.is_cuda:
        logits = F.linear(x.float(), wte)
        return F.cross_entropy(logits.reshape(-1, logits.shape[-1]), labels.reshape(-1), ignore_index=ignore_index)
    V = wte.shape[0]
    Vp = (V + vocab_pad_to - 1) // vocab_pad_to * vocab_pad_to
    return _LMHeadCEFn.apply(x, wte, labels, Vp - V, ignore_index)


def lm_head(x, wte, vocab_pad_to: int = 64):
    V = wte.shape[0]
    Vp = (V + vocab_pad_to - 1) // vocab_pad_to * vocab_pad_to
    if not x.is_cuda:
        return F.linear(x.float(), wte)
    return _LMHeadFn.apply(x, wte, Vp - V)
