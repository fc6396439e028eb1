"""SimpleNet -- the reference's model (`train.py:32-50`), same structure,
same parameter names/shapes (``layers.{0,3,6}.{weight,bias}``, 269,322
parameters) so checkpoints interchange with the reference.  On the GPU each
Linear runs the gfx950 MFMA GEMM with the bias+ReLU fused into its epilogue
(SURVEY §2.6.1 K2-K8).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops import functional as Fx
from ..ops.layers import Dropout, Flatten, Linear, ReLU


class SimpleNet(nn.Module):
    def __init__(self, input_size: int = 784, hidden_size: int = 256, num_classes: int = 10):
        super().__init__()
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
        if x.is_cuda:
            # fused epilogues: Linear+bias+ReLU in one GEMM launch
            h = Fx.linear(x, l0.weight, l0.bias, Fx.ACT_RELU)
            h = d0(h)
            h = Fx.linear(h, l1.weight, l1.bias, Fx.ACT_RELU)
            h = d1(h)
            return l2(h)
        return self.layers(x)
