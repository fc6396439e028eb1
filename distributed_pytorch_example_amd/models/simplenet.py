"""SimpleNet -- the reference's model (`train.py:32-50`), same structure,
same parameter names/shapes (``layers.{0,3,6}.{weight,bias}``, 269,322
parameters) so checkpoints interchange with the reference.

GPU paths (``compute_dtype``):

* ``"fp32"`` (default: the reference trains in fp32, `train.py:249`): the whole
  network is one autograd node on the exact-f32 MFMA GEMM
  (csrc/kernels/gemm_f32.hip) -- bias + ReLU + Dropout(0.2) fused into each
  hidden GEMM's epilogue (Philox mask, identical to the standalone dropout
  kernel for the same (seed, offset)); backward fuses each ReLU+dropout
  backward into the data-grad epilogue of the layer above (``y > 0`` of the
  saved output is exactly "kept and positive"), weight gradients go straight
  into the DDP bucket views.
* ``"bf16"``: bf16 MFMA GEMMs with bias+ReLU fused, standalone Philox dropout.
"""
from __future__ import annotations

import torch
import torch.nn as nn
from torch.autograd import Function

from ..ops import functional as Fx
from ..ops._ext import ext
from ..ops._state import grad_done, grad_sink, note_use
from ..ops.layers import Dropout, Flatten, Linear, ReLU


class _SimpleNet32Fn(Function):
    @staticmethod
    def forward(ctx, x, p0: float, p1: float, training: bool, w0, b0, w1, b1, w2, b2):
        C = ext()
        h = x.reshape(x.shape[0], -1)
        h = (h if h.dtype == torch.float32 else h.float()).contiguous()
        acts = [h]
        scales = []
        for w, b, p in ((w0, b0, p0), (w1, b1, p1)):  # each hidden layer's own Dropout(p)
            drop = training and p > 0.0
            seed, off = Fx._RNG.next(h.shape[0] * w.shape[0]) if drop else (0, 0)
            h = C.linear32_fwd(h, w.detach(), b.detach(), True, p if drop else 0.0, seed, off)
            acts.append(h)
            scales.append(1.0 / (1.0 - p) if drop else 1.0)
        logits = C.linear32_fwd(h, w2.detach(), b2.detach())
        ctx.save_for_backward(*acts)
        ctx.params = (w0, b0, w1, b1, w2, b2)
        ctx.scales = tuple(scales)
        ctx.xshape = x.shape
        for t in ctx.params:
            note_use(t)
        return logits

    @staticmethod
    def backward(ctx, g):
        C = ext()
        x, y0, y1 = ctx.saved_tensors
        w0, b0, w1, b1, w2, b2 = ctx.params
        g = g.contiguous().float()

        def wgrad(w, dy, inp):
            buf, direct = grad_sink(w)
            C.linear32_wgrad(dy, inp, buf, 1.0)
            grad_done(w, direct)
            return None if direct else buf

        def bgrad(b, dy):
            buf, direct = grad_sink(b)
            C.colsum(dy, buf, True)
            grad_done(b, direct)
            return None if direct else buf

        gw2, gb2 = wgrad(w2, g, y1), bgrad(b2, g)
        s0, s1 = ctx.scales
        dh1 = C.linear32_dgrad(g, w2.detach(), y1, s1)   # relu+dropout(p1) backward of layer 1 fused
        gw1, gb1 = wgrad(w1, dh1, y0), bgrad(b1, dh1)
        dh0 = C.linear32_dgrad(dh1, w1.detach(), y0, s0)
        gw0, gb0 = wgrad(w0, dh0, x), bgrad(b0, dh0)
        dx = C.linear32_dgrad(dh0, w0.detach()).reshape(ctx.xshape) if ctx.needs_input_grad[0] else None
        return dx, None, None, None, gw0, gb0, gw1, gb1, gw2, gb2


class SimpleNet(nn.Module):
    def __init__(self, input_size: int = 784, hidden_size: int = 256, num_classes: int = 10,
                 compute_dtype: str = "fp32"):
        super().__init__()
        if compute_dtype not in ("fp32", "bf16"):
            raise ValueError(f"compute_dtype must be 'fp32' or 'bf16', got {compute_dtype!r}")
        self.compute_dtype = compute_dtype
        self.flatten = Flatten()
        self.layers = nn.Sequential(
            Linear(input_size, hidden_size),
            ReLU(),
            Dropout(0.2),
            Linear(hidden_size, hidden_size),
            ReLU(),
            Dropout(0.2),
            Linear(hidden_size, num_classes, out_f32=True),
        )

    def forward(self, x):
        x = self.flatten(x)
        l0, _, d0, l1, _, d1, l2 = self.layers
        if x.is_cuda and self.compute_dtype == "fp32":
            return _SimpleNet32Fn.apply(x, d0.p, d1.p, self.training, l0.weight, l0.bias, l1.weight, l1.bias, l2.weight,
                                        l2.bias)
        if x.is_cuda:
            # bf16: fused epilogues, Linear+bias+ReLU in one GEMM launch
            h = Fx.linear(x, l0.weight, l0.bias, Fx.ACT_RELU)
            h = d0(h)
            h = Fx.linear(h, l1.weight, l1.bias, Fx.ACT_RELU)
            h = d1(h)
            return l2(h)
        return self.layers(x)
