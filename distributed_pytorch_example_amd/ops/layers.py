"""nn.Module layers over the ops in ``functional``.

Parameters are fp32 masters with torch-compatible names and shapes where the
reference's checkpoints depend on them (Linear: ``weight [out, in]``,
``bias [out]``).  Conv filters are stored OHWI (``[out, kh, kw, in]``) -- the
layout the gfx950 implicit GEMM reads K-contiguously.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import functional as Fx


class Linear(nn.Module):
    def __init__(self, in_features: int, out_features: int, bias: bool = True, act: int = Fx.ACT_NONE,
                 out_f32: bool = False, device=None):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.act, self.out_f32 = act, out_f32
        self.weight = nn.Parameter(torch.empty(out_features, in_features, device=device))
        self.bias = nn.Parameter(torch.empty(out_features, device=device)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        # same init as torch.nn.Linear
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            bound = 1 / math.sqrt(self.in_features) if self.in_features > 0 else 0
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x):
        return Fx.linear(x, self.weight, self.bias, self.act, self.out_f32)

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}, bias={self.bias is not None}"


class ReLU(nn.Module):
    def forward(self, x):
        return Fx.relu(x)


class GELU(nn.Module):
    def forward(self, x):
        return Fx.gelu(x)


class Dropout(nn.Module):
    def __init__(self, p: float = 0.5):
        super().__init__()
        self.p = p

    def forward(self, x):
        return Fx.dropout(x, self.p, self.training)

    def extra_repr(self):
        return f"p={self.p}"


class Flatten(nn.Module):
    def forward(self, x):
        return x.reshape(x.shape[0], -1)


class Conv2d(nn.Module):
    """NHWC convolution, filter stored [out, kh, kw, in]."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, bias=False,
                 device=None):
        super().__init__()
        k = Fx._pair(kernel_size)
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size, self.stride, self.padding, self.dilation = k, Fx._pair(stride), Fx._pair(padding), Fx._pair(dilation)
        self.weight = nn.Parameter(torch.empty(out_channels, k[0], k[1], in_channels, device=device))
        if bias:
            raise NotImplementedError("Conv2d bias: use a following BatchNorm (ResNet) or a Linear")
        self.reset_parameters()

    def reset_parameters(self):
        # kaiming_normal_(mode='fan_out', nonlinearity='relu') as torchvision ResNet
        fan_out = self.out_channels * self.kernel_size[0] * self.kernel_size[1]
        std = math.sqrt(2.0 / fan_out)
        with torch.no_grad():
            self.weight.normal_(0, std)

    def forward(self, x, want_stats: bool = False):
        return Fx.conv2d_nhwc(x, self.weight, self.stride, self.padding, self.dilation, want_stats)

    def extra_repr(self):
        return (f"{self.in_channels}, {self.out_channels}, kernel_size={self.kernel_size}, stride={self.stride}, "
                f"padding={self.padding}, layout=NHWC/OHWI")


class BatchNorm2d(nn.Module):
    """BatchNorm over the channel (last) dim of NHWC activations, optional fused ReLU / residual add."""

    def __init__(self, num_features: int, eps: float = 1e-5, momentum: float = 0.1, device=None):
        super().__init__()
        self.num_features, self.eps, self.momentum = num_features, eps, momentum
        self.weight = nn.Parameter(torch.ones(num_features, device=device))
        self.bias = nn.Parameter(torch.zeros(num_features, device=device))
        self.register_buffer("running_mean", torch.zeros(num_features, device=device))
        self.register_buffer("running_var", torch.ones(num_features, device=device))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long, device=device))

    def forward(self, x, relu: bool = False, residual=None, stats=None):
        return Fx.batch_norm_nhwc(x, self.weight, self.bias, self.running_mean, self.running_var, self.training,
                                  self.momentum, self.eps, relu, residual, stats, self.num_batches_tracked)


class LayerNorm(nn.Module):
    def __init__(self, dim: int, eps: float = 1e-5, bias: bool = True, device=None):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim, device=device))
        self.bias = nn.Parameter(torch.zeros(dim, device=device)) if bias else None

    def forward(self, x):
        return Fx.layer_norm(x, self.weight, self.bias, self.eps)


class CrossEntropyLoss(nn.Module):
    """torch.nn.CrossEntropyLoss (mean) on the fused HIP kernel."""

    def __init__(self, ignore_index: int = -100):
        super().__init__()
        self.ignore_index = ignore_index

    def forward(self, logits, target):
        return Fx.cross_entropy(logits, target, None, self.ignore_index)
