"""ResNet-50 v1.5 (BASELINE.json configs 2, 3, 5) in NHWC for gfx950.

Topology is torchvision's ``resnet50`` (stride on the 3x3 conv, 25,557,032
parameters, zero-init of nothing) -- SURVEY §2.6.2 lists its 23 conv shapes.
Execution is MI355X-native:

* activations NHWC bf16, filters OHWI (implicit-GEMM K-contiguous);
* every conv feeding a BatchNorm accumulates that BN's per-channel
  (sum, sum^2) in its GEMM epilogue, so the BN statistics pass is skipped;
* BN apply fuses ReLU and the residual add (one pass per BN);
* the 7x7/s2 stem runs as a 4x4/s1 conv over a space-to-depth packed input
  ([N,112,112,16]: 35% fewer MFMA k-steps than an 8-channel-padded 7x7);
  its BN + ReLU are applied inside the max-pool (never materialised);
* each block's BN3 backward is fused into the next block's data-grad
  epilogue (``_resnet_fused``).
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.nn as nn

from ..ops import functional as Fx
from ..ops.layers import BatchNorm2d, Conv2d, Linear


class ConvBN(nn.Module):
    """conv -> BN (training stats from the conv epilogue) -> optional residual add -> optional ReLU."""

    def __init__(self, cin, cout, k, stride=1, padding=0):
        super().__init__()
        self.conv = Conv2d(cin, cout, k, stride, padding)
        self.bn = BatchNorm2d(cout)

    def forward(self, x, relu=True, residual=None):
        if self.bn.training and x.is_cuda:
            y, st = self.conv(x, want_stats=True)   # BN statistics from the conv epilogue
        else:
            y, st = self.conv(x), None
        return self.bn(y, relu=relu, residual=residual, stats=st)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=False):
        super().__init__()
        width = planes
        self.c1 = ConvBN(inplanes, width, 1)
        self.c2 = ConvBN(width, width, 3, stride, 1)
        self.c3 = ConvBN(width, planes * 4, 1)
        self.down = ConvBN(inplanes, planes * 4, 1, stride) if downsample else None
        cbs = [self.c1, self.c2, self.c3] + ([self.down] if downsample else [])
        self._fused_params = [t for cb in cbs for t in (cb.conv.weight, cb.bn.weight, cb.bn.bias)]
        self.fused = True

    def forward(self, x):
        return self.forward_chained(x, None, chain=False)

    def forward_chained(self, x, link=None, chain=True, count_batches=True, defer_out=False, gram_next=0):
        """``chain=True``: returns (out, link); the link lets the next block's
        backward fuse this block's BN3 backward (``_resnet_fused``).
        ``count_batches=False``: the caller already advanced the BNs' num_batches_tracked.
        ``defer_out``: the output is written by the next block's conv1 (called next)."""
        if x.is_cuda and self.training and self.fused:
            from ._resnet_fused import bottleneck_forward

            return bottleneck_forward(self, x, link, chain, count_batches, defer_out, gram_next)
        out = self._forward_per_op(x)
        return (out, None) if chain else out

    def _forward_per_op(self, x):
        idn = self.down(x, relu=False) if self.down is not None else x
        h = self.c1(x)
        h = self.c2(h)
        return self.c3(h, relu=True, residual=idn)


class ResNet(nn.Module):
    def __init__(self, layers: List[int] = (3, 4, 6, 3), num_classes: int = 1000, in_chans: int = 3, in_pad: int = 8):
        super().__init__()
        self.in_pad = in_pad
        # GPU: 7x7/s2 stem as a 4x4/s1 conv over a space-to-depth input (DPE_S2D_STEM=0: NHWC-8 stem)
        self.s2d_stem = in_chans <= 4 and os.environ.get("DPE_S2D_STEM", "1") != "0"
        # GPU training: stem BN + ReLU fused into the max-pool (DPE_FUSED_STEM=0: separate passes)
        self.fused_stem = os.environ.get("DPE_FUSED_STEM", "1") != "0"
        # GPU training: the whole stem as one node whose backward never writes dL/dh (DPE_STEM_BWD_FUSED=0: the
        # BN / max-pool backward as its own apply pass, A/B)
        self.stem_bwd_fused = self.fused_stem and os.environ.get("DPE_STEM_BWD_FUSED", "1") != "0"
        self.stem = ConvBN(in_chans, 64, 7, 2, 3)
        blocks = []
        inplanes = 64
        for i, (n, planes) in enumerate(zip(layers, (64, 128, 256, 512))):
            for j in range(n):
                stride = 2 if (j == 0 and i > 0) else 1
                blocks.append(Bottleneck(inplanes, planes, stride, downsample=(j == 0)))
                inplanes = planes * 4
        self.blocks = nn.Sequential(*blocks)
        self.fc = Linear(512 * 4, num_classes, out_f32=True)

    def forward(self, x):
        """x: NCHW float images [N,3,H,W], or packed on the GPU: space-to-depth
        [N,H/2,W/2,16] bf16 (``Fx.to_s2d_input``) or NHWC [N,H,W,in_pad]."""
        if x.is_cuda and self.s2d_stem:
            if x.dim() == 4 and x.shape[1] == 3:
                x = Fx.to_s2d_input(x)
            elif x.shape[-1] == self.in_pad and self.in_pad >= 4:  # NHWC-packed -> s2d (view shuffle)
                n, hh, ww, _ = x.shape
                x = x[..., :4].reshape(n, hh // 2, 2, ww // 2, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(
                    n, hh // 2, ww // 2, 16)
            bn = self.stem.bn
            if bn.training and self.stem_bwd_fused and Fx.stem_fused_ok(x):
                h = Fx.stem_fused(x, self.stem.conv.weight, bn)
            elif bn.training and self.fused_stem:
                # BN statistics from the conv epilogue; BN + ReLU applied inside the max-pool
                y, st = Fx.stem_conv_s2d(x, self.stem.conv.weight, want_stats=True)
                h = Fx.stem_bn_relu_maxpool(y, bn, st, 3, 2, 1)
            else:
                if bn.training:
                    y, st = Fx.stem_conv_s2d(x, self.stem.conv.weight, want_stats=True)
                else:
                    y, st = Fx.stem_conv_s2d(x, self.stem.conv.weight), None
                h = Fx.max_pool2d_nhwc(bn(y, relu=True, stats=st), 3, 2, 1)
        else:
            if x.dim() == 4 and x.shape[1] != self.in_pad and x.shape[-1] != self.in_pad:
                x = Fx.to_nhwc_input(x, self.in_pad)
            h = Fx.max_pool2d_nhwc(self.stem(x), 3, 2, 1)
        link = None
        # the blocks that take the fused path (the same test forward_chained makes per block): their
        # num_batches_tracked counters advance in one multi-tensor launch instead of one per block;
        # the list is rebuilt per step (host-side only) so moved / reloaded buffers are never stale
        fused = [h.is_cuda and self.training and b.training and b.fused for b in self.blocks]
        if any(fused):
            torch._foreach_add_([m.num_batches_tracked for b, f in zip(self.blocks, fused) if f for m in b.modules()
                                 if getattr(m, "num_batches_tracked", None) is not None], 1)
        # a block's output may be left to the next block's conv1 to write (on-load BN3 apply)
        defer = [False] * len(fused)
        if any(fused):
            from ._resnet_fused import can_materialise_input

            defer = [f and i + 1 < len(fused) and fused[i + 1] and can_materialise_input(self.blocks[i + 1])
                     for i, f in enumerate(fused)]
        # BN3 by Gram algebra (no h3 tensor, no BN3 apply passes) where the next block can chain its backward
        gram = [0] * len(fused)
        if any(fused):
            from ._resnet_fused import gram_successor_width

            gram = [gram_successor_width(self.blocks[i + 1]) if (f and i + 1 < len(fused) and fused[i + 1]) else 0
                    for i, f in enumerate(fused)]
        for blk, f, d, gn in zip(self.blocks, fused, defer, gram):  # each block's output feeds only the next block
            h, link = blk.forward_chained(h, link, count_batches=not f, defer_out=d, gram_next=gn)
        h = Fx.global_avg_pool_nhwc(h)
        return self.fc(h)


def resnet50(num_classes: int = 1000) -> ResNet:
    return ResNet((3, 4, 6, 3), num_classes)


def resnet18_like(num_classes: int = 10) -> ResNet:
    """Small bottleneck ResNet for fast tests."""
    return ResNet((1, 1, 1, 1), num_classes)
