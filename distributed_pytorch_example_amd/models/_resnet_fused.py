"""Hand-scheduled forward/backward of a ResNet bottleneck block on gfx950.

One autograd node per block instead of ~12 per-op nodes:

forward  (x NHWC bf16)
    [hd = conv_d(x)]                                             (downsample blocks)
    h1 = conv1(x)  -> a1 = relu(BN1(h1))      BN statistics come from the conv epilogue
    h2 = conv2(a1) -> a2 = relu(BN2(h2))
    h3 = conv3(a2) -> out = relu(BN3(h3) + idn)    idn = x, or BN_d(hd) computed inside
                                                   the same pass (never stored)
backward (dout)
    dh3, dz3 = BN3'(dout; out, h3)            dz3 = dout*relu'(out) is also d(idn)
    dW3 += dh3 (x) a2 ;  da2 = dh3 . W3       the dgrad epilogue also emits BN2's backward
                                              sums (sum dz, sum dz*(h2-mean)), ReLU mask from h2
    dh2 = BN2'(da2; h2)                       one elementwise pass: no separate reduce pass over da2
    dW2 += dh2 (x) a1 ; da1 = dh2 . W2 (+ BN1 sums) ; dh1 = BN1'(da1; h1) ; dW1 += dh1 (x) x
    identity block:   dx = dh1 . W1 + dz3            (residual add fused in the dgrad epilogue)
    downsample block: dhd = BN_d'(dz3; hd); dW_d += dhd (x) x
                      dx = dh1 . W1 ; dx += dhd . W_d   (in place, only the parity the strided
                                                         1x1 reaches is touched)

Cross-block fusion of BN3's backward (DPE_BN3_CHAIN=1, default): block i's
output ``out_i`` is consumed only by block i+1.  When block i+1 is an identity
block, the epilogue of its first data-grad (dx = dh1 . W1 + dz3) also applies
block i's ReLU mask (out_i > 0, i.e. relu'(BN3_i(h3_i) + idn_i); read as the
bit mask that block i's BN3 apply wrote beside out_i -- 1/16 of out_i's
bytes), stores the masked dz3_i directly, and emits BN3_i's backward partials (sum dz, sum
dz*(h3_i - mean)).  Block i's BN3 backward is then ONE elementwise pass
(dh3 = a*dz3 + b*h3 + c) instead of a reduce pass over (dout, out, h3) plus an
apply pass that re-reads all three and writes dz3: three fewer full passes
over the block's widest tensor.  The hand-off is a ``_BN3Link`` object filled
by block i's forward and consumed by block i+1; if the gradient block i
receives is not the tensor that epilogue produced, block i falls back to the
standalone path (masking an already-masked gradient again is idempotent).

(A variant that also fused BN1/BN2 + ReLU into the implicit-GEMM convs' load
prologues, never materialising a1/a2, measured slower on MI355X: the
transform sits on the loaders' critical path and the inner BN tensors carry
only 1/4 of the block's channels -- so those outputs are materialised.  The
exception is a1 of the 64-channel layer-1 blocks (DPE_ROW_BNIN=1, default):
conv2 and its weight grad run on the row-walking kernels (rowconv.hip), which
stage every input row through registers one row ahead of its use, so
relu(BN1(h1)) is applied there off the critical path and a1 (205 MB at batch
512) is neither written nor re-read: conv2 reads h1 + BN1's coefficients, the
weight grad recomputes a1 the same way, and BN1's backward already takes its
ReLU mask from h1.  Likewise a2 (DPE_PW_BNIN=1, default): the streaming
pointwise conv3 forward and its LDS-DMA weight grad apply relu(BN2(h2)) to
their operand fragments.)

Block outputs and BN3 backward applies on load (DPE_AX_FWD=1 / DPE_AX_BWD=1): block i's
output out_i = relu(BN3(h3_i) + idn_i) is not written by a bn_apply pass of its own.  Block i+1's
conv1 (1x1, stride 1) computes it on its A fragments from (h3_i, idn_i) and BN3_i's coefficients
and stores it once as a by-product (with its ReLU-mask bits) for the consumers that need it later
(block i+1's identity / downsample conv, its conv1 weight grad, the backward masks): the pass that
wrote out_i read the same two tensors, so conv1's own read of out_i is what disappears.  In
backward, block i's dh3 = a*dz3 + b*h3 + c is likewise computed on the A fragments of conv3's data
grad and stored once for conv3's weight grad (conv1x1_bnin_fwd / conv1x1_bnin_dgrad, igemm.hip
AXform).  That removes one full read of each such tensor.  Measured: the backward form pays in
layers 1-2 (default there), the forward form does not (off by default; see the flags below).

Weight gradients are accumulated straight into the DDP bucket views and each
parameter is announced to the reducer as soon as its gradient is final, in
reverse-forward order, so bucket all-reduces start while earlier blocks are
still in backward.
"""
from __future__ import annotations

import os

import torch
from torch.autograd import Function

from ..ops._ext import ext
from ..ops._state import finalize_stream, grad_done, grad_sink, note_use, run_on_aux, shadow

# DPE_BN_EPI=0: inner BN backward through the standalone reduce kernel (A/B reference)
_EPI_BNB = os.environ.get("DPE_BN_EPI", "1") != "0"
# DPE_BN3_CHAIN=0: every block's BN3 backward through the standalone reduce + apply
_BN3_CHAIN = _EPI_BNB and os.environ.get("DPE_BN3_CHAIN", "1") != "0"
# DPE_BN_DUAL=0: downsample blocks run BN3's and BN_d's backward as separate passes
_BN_DUAL = os.environ.get("DPE_BN_DUAL", "1") != "0"
# DPE_ROW_BNIN=0: layer-1 a1 = relu(BN1(h1)) materialised by a bn_apply pass (A/B reference)
_ROW_BNIN = _EPI_BNB and os.environ.get("DPE_ROW_BNIN", "1") != "0"
# DPE_PW_BNIN=0: layer-1 a2 = relu(BN2(h2)) materialised by a bn_apply pass (A/B reference)
_PW_BNIN = _EPI_BNB and os.environ.get("DPE_PW_BNIN", "1") != "0"
# DPE_DOWN_CHAIN=0: the block before a downsample block runs its BN3 backward standalone (reduce + apply)
_DOWN_CHAIN = _BN3_CHAIN and os.environ.get("DPE_DOWN_CHAIN", "1") != "0"
# DPE_AX_FWD=1: block outputs written by the next block's conv1 instead of a bn_apply pass.  Off:
# measured slower at every ResNet-50 shape (scripts/bench_bnin.py, profiles/bnin_r3.jsonl: layer 1
# 654 vs 635 us, layers 3-4 +20-80 %) -- the by-product leaves the K-loop in 64-B row segments
# (one 32-deep K-step per row per store), which the memory system absorbs at ~3 TB/s where the
# streaming pass writes whole 1-KiB runs at ~6 TB/s.
_AX_FWD = _BN3_CHAIN and os.environ.get("DPE_AX_FWD", "0") == "1"
# DPE_AX_BWD=1: every chained block's dh3 (of at most DPE_AX_BWD_MAXC channels) computed on conv3's
# data-grad fragments instead of a bn_bwd_apply pass.  Per op: layer 2 -11 %, layer 1 -1.5 %,
# layers 3-4 +1-19 % (profiles/bnin_r3.jsonl); on the ResNet-50 step within noise (37.99-38.15 vs
# 37.99-38.11 ms, 3 alternating rounds), so off by default -- kept as a tested building block.
_AX_BWD = _BN3_CHAIN and os.environ.get("DPE_AX_BWD", "0") == "1"
_AX_BWD_MAXC = int(os.environ.get("DPE_AX_BWD_MAXC", "512"))
# row tile of the on-load forward at 64 output channels (128: 4 blocks/CU, 256: 2; the
# downsample-identity form spills at 128)
_AX_TILE = int(os.environ.get("DPE_AX_TILE", "256"))
# DPE_BN3_GRAM=1: BN3 by Gram algebra (csrc/kernels/bngram.hip).  h3 = a2 W3^T is linear in a2, so BN3's
# statistics come from G = a2^T a2 and s = colsum(a2) BEFORE conv3 runs: conv3's epilogue writes the
# block output relu(BN3(h3) + idn) directly (no h3 tensor, no bn_apply pass), and the backward needs
# neither h3 nor dh3 (dW3 = diag(a) dz3^T a2 + diag(b) W3 G + c s^T; da2 = [dz3 | a2] x [diag(a) W3 ; Q]),
# so there is no bn_bwd_apply pass and the next block's data-grad epilogue reads no h3.  For blocks whose
# conv3 runs on the streaming pointwise kernel and whose successor chains BN3's backward.
_GRAM = _BN3_CHAIN and os.environ.get("DPE_BN3_GRAM", "1") != "0"


def _ax_ok(conv, cin) -> bool:
    """A 1x1 stride-1 conv whose input channels the on-load transform kernel takes."""
    return (tuple(conv.kernel_size) == (1, 1) and tuple(conv.stride) == (1, 1) and tuple(conv.padding) == (0, 0)
            and cin % 32 == 0 and cin <= 2048)


def can_materialise_input(block) -> bool:
    """True when ``block``'s conv1 can compute (and store) its input from the previous block's
    pre-BN3 tensors, so the previous block may defer its output (DPE_AX_FWD)."""
    return _AX_FWD and block.fused and _ax_ok(block.c1.conv, block.c1.conv.in_channels)


def _out_hw(hw, conv):
    k, s, p, d = conv.kernel_size[0], conv.stride[0], conv.padding[0], conv.dilation[0]
    return (hw + 2 * p - d * (k - 1) - 1) // s + 1


class _BN3Link:
    """Block i's (h3, BN3 coefficients) handed to block i+1, and block i+1's
    fused-epilogue result (BN3_i partials, identity of the masked dz3_i)
    handed back to block i's backward."""

    __slots__ = ("h3", "coef", "mask", "part", "dz_ptr", "dz_shape", "pending", "gram")

    def __init__(self):
        self.h3 = self.coef = self.mask = self.part = None
        self.dz_ptr, self.dz_shape = 0, None
        self.gram = False  # block i ran BN3 by Gram algebra: block i+1's epilogue emits only the sum-dz partials
        # (h3, coef3, idn, idn_coef, out, bits): block i's output, allocated but not yet written --
        # block i+1's conv1 writes it (conv1x1_bnin_fwd)
        self.pending = None


def _conv_conf(conv):
    return list(conv.stride), list(conv.padding), list(conv.dilation)


class BottleneckFn(Function):
    @staticmethod
    def forward(ctx, x, block, link_in, link_out, defer_out, gram_next, *params):
        C = ext()
        convs = [block.c1, block.c2, block.c3] + ([block.down] if block.down is not None else [])
        ws = [shadow(cb.conv.weight) for cb in convs]
        pend = link_in.pending if link_in is not None else None
        if pend is not None:
            # x is the previous block's output, not yet written: conv1 computes it on load from
            # (h3, identity) and BN3's coefficients and stores it (+ its ReLU bits) as a by-product
            ph3, pc3, pidn, pcd, pout, pbits = pend
            assert pout is x, "deferred block output consumed by a different tensor"
            link_in.pending = None
            h1_st = C.conv1x1_bnin_fwd(ph3, pidn, pc3, pcd, ws[0], x, pbits, True, _AX_TILE)
        else:
            h1_st = None

        def convbn(i, inp, relu, residual=None):
            cb = convs[i]
            s, p, d = _conv_conf(cb.conv)
            if i == 0 and h1_st is not None:
                h, st = h1_st
            else:
                h, st = C.conv_fwd(inp, ws[i], s, p, d, True, None)  # BN stats partials from the epilogue
            bn = cb.bn
            y, coef = C.bn_fwd_train(h, bn.weight.detach(), bn.bias.detach(), bn.running_mean, bn.running_var,
                                     bn.momentum, bn.eps, relu, residual, st)
            return h, y, coef

        def conv_coef(i, inp, in_coef=None):
            cb = convs[i]
            s, p, d = _conv_conf(cb.conv)
            if i == 0 and h1_st is not None:
                h, st = h1_st
            else:
                h, st = C.conv_fwd(inp, ws[i], s, p, d, True, None, in_coef)
            bn = cb.bn
            M = h.numel() // h.shape[-1]
            return h, C.bn_coef(st, M, bn.weight.detach(), bn.bias.detach(), bn.running_mean, bn.running_var, bn.momentum,
                                bn.eps)

        c1conv, c2conv = convs[0].conv, convs[1].conv
        if h1_st is None and block.down is not None:
            hd, cd = conv_coef(3, x)  # BN_d is applied inside BN3's pass (bn_apply with residual_coef)
        else:
            hd, cd = None, None  # (x still pending: after conv1 has written it)
        h1_shape = [x.shape[0], _out_hw(x.shape[1], c1conv), _out_hw(x.shape[2], c1conv), c1conv.out_channels]
        if _ROW_BNIN and C.row_bn_on_load(h1_shape, list(ws[1].shape), *_conv_conf(c2conv)):
            # a1 never materialised: conv2 applies relu(BN1(h1)) to its input rows on load
            h1, c1 = conv_coef(0, x)
            a1 = None
            h2, st2 = C.conv_fwd(h1, ws[1], *_conv_conf(c2conv), True, None, c1)
        else:
            h1, a1, c1 = convbn(0, x, True)
            h2, st2 = C.conv_fwd(a1, ws[1], *_conv_conf(c2conv), True, None)
        if h1_st is not None and block.down is not None:
            hd, cd = conv_coef(3, x)  # x written by conv1 above
        bn2 = convs[1].bn
        if _PW_BNIN and C.pw_bn_on_load(list(h2.shape), convs[2].conv.out_channels):
            # a2 never materialised: the streaming conv3 forward and its LDS-DMA weight grad apply
            # relu(BN2(h2)) to their operand fragments (64- and 128-channel bottlenecks)
            c2 = C.bn_coef(st2, h2.numel() // h2.shape[-1], bn2.weight.detach(), bn2.bias.detach(),
                           bn2.running_mean, bn2.running_var, bn2.momentum, bn2.eps)
            a2 = None
        else:
            a2, c2 = C.bn_fwd_train(h2, bn2.weight.detach(), bn2.bias.detach(), bn2.running_mean,
                                    bn2.running_var, bn2.momentum, bn2.eps, True, None, st2)
        # the next block's fused data-grad epilogue reads this output's ReLU mask as bits
        want_bits = True  # 1/16 of out: read by the next block's fused epilogue or by this block's BN3 backward
        gram = None
        # gram_next < 0: the successor is a downsample block, which chains this block's BN3 backward only
        # when its strided conv1 data grad can take the residual (the successor's own strided_ok test)
        out_shape = [*h2.shape[:3], convs[2].conv.out_channels]
        if (gram_next and link_out is not None and not defer_out and h1_st is None
                and (gram_next > 0 or C.pw_dgrad_strided_residual_ok(out_shape, -gram_next))
                and C.gram_ok(list(h2.shape), convs[2].conv.out_channels, abs(gram_next))):
            # BN3 statistics from G = a2^T a2, s = colsum(a2); conv3 writes relu(BN3(h3) + idn) directly
            src, src_coef = (h2, c2) if a2 is None else (a2, None)
            G, sv = C.bn_gram(src, src_coef, c2)  # centred on a pilot shift from BN2's coefficients
            bn3 = convs[2].bn
            M3 = h2.numel() // h2.shape[-1]
            c3, u3 = C.bn_gram_coef(G, sv, ws[2], M3, bn3.weight.detach(), bn3.bias.detach(), bn3.running_mean,
                                    bn3.running_var, bn3.momentum, bn3.eps)
            if block.down is not None:
                out, bits = C.conv1x1_apply(src, ws[2], src_coef, c3, hd, cd)
            else:
                out, bits = C.conv1x1_apply(src, ws[2], src_coef, c3, x, None)
            h3 = None
            gram = (u3, sv, M3)
        else:
            h3, c3 = conv_coef(2, h2, c2) if a2 is None else conv_coef(2, a2)
        if gram is not None:
            pass
        elif defer_out and link_out is not None:
            # written later by the next block's conv1 (conv1x1_bnin_fwd): no bn_apply pass
            out = torch.empty_like(h3)
            bits = torch.empty(*h3.shape[:-1], h3.shape[-1] // 8, dtype=torch.uint8, device=h3.device)
            link_out.pending = (h3, c3, hd, cd, out, bits) if block.down is not None else (h3, c3, x, None, out, bits)
        elif block.down is not None:
            out, bits = C.bn_apply(h3, c3, hd, cd, True, want_bits)
        else:
            out, bits = C.bn_apply(h3, c3, x, None, True, want_bits)
        ctx.save_for_backward(x, h1, a1, h2, a2, h3, out, hd, c1, c2, c3, cd)
        # previous block's BN3 is fused into this block's first data grad.  A downsample block's dx also
        # has the stride-2 branch's term: it is computed first as a compact [N, H/2, W/2, C] data grad
        # and added at the even pixels by the streaming conv1 data grad's epilogue, which then applies
        # the mask and emits the partials as for an identity block (layers 1 -> 2 and 2 -> 3).
        strided_ok = block.down is not None and _DOWN_CHAIN and tuple(block.down.conv.stride) == (2, 2) and \
            tuple(block.down.conv.kernel_size) == (1, 1) and tuple(convs[0].conv.stride) == (1, 1) and \
            C.pw_dgrad_strided_residual_ok(list(x.shape), convs[0].conv.out_channels)
        ctx.link_in = (link_in if (link_in is not None and (block.down is None or strided_ok)
                                   and (link_in.h3 is not None or link_in.gram) and link_in.mask is not None) else None)
        if link_in is not None and link_in.gram and ctx.link_in is None:
            # the previous block has no h3 and no standalone BN3 backward: this block must chain it
            # (gram_successor_width + the strided test above make this unreachable; fail loudly if not)
            raise RuntimeError("BN3 Gram path: the next block cannot chain the BN3 backward "
                               f"(input {tuple(x.shape)}, downsample={block.down is not None})")
        ctx.link_out = link_out
        ctx.bits = bits  # ReLU mask of out as bits: the standalone BN3 backward reads these, not out
        ctx.gram = gram
        if link_out is not None:
            link_out.h3, link_out.coef, link_out.mask = h3, c3, bits
            link_out.gram = gram is not None
            if gram is not None and block.down is not None:
                # the next block's data-grad epilogue reduces the downsample BN's partials instead
                # (sum dz, sum dz*(hd - mean_d)): row 0 serves BN3's Gram backward, both rows BN_d's
                link_out.h3, link_out.coef = hd, cd
        ctx.block = block
        ctx.convs = convs
        ctx.ws = ws
        for cb in convs:
            note_use(cb.conv.weight)
            note_use(cb.bn.weight)
            note_use(cb.bn.bias)
        return out

    @staticmethod
    def backward(ctx, dout):
        C = ext()
        x, h1, a1, h2, a2, h3, out, hd, c1, c2, c3, cd = ctx.saved_tensors
        convs, ws = ctx.convs, ctx.ws
        has_down = len(convs) == 4
        dout = dout.contiguous()
        grads = {}
        res_mask = None  # set when dz3 is represented as (dout, ReLU bits of out)
        dhd = None  # downsample BN's dL/dhd, when computed together with BN3's (bn_bwd_dual)
        dh3_coef = None  # set when dh3 is computed on load by conv3's data grad

        def bn_sinks(i):
            bn = convs[i].bn
            gb, gd = grad_sink(bn.weight)
            bb, bd = grad_sink(bn.bias)
            return bn, gb, gd, bb, bd

        def bn_done(bn, gb, gd, bb, bd):
            grad_done(bn.weight, gd)
            grad_done(bn.bias, bd)
            grads[id(bn.weight)] = None if gd else gb
            grads[id(bn.bias)] = None if bd else bb

        def bn_bwd(i, dy, y, h, coef, want_dz, y_bits=None):
            bn, gb, gd, bb, bd = bn_sinks(i)
            dh, dz = C.bn_bwd(dy, y, h, bn.weight.detach(), coef, gb, bb, want_dz, y_bits)
            bn_done(bn, gb, gd, bb, bd)
            return dh, dz

        def wgrad(i, dy, inp, in_coef=None):
            w = convs[i].conv.weight
            s, p, d = _conv_conf(convs[i].conv)
            buf, direct = grad_sink(w)
            if direct:  # bucket view: on the weight-grad side stream (the reducers wait for it)
                fs = finalize_stream(dy.device)  # a K-split hgemm's slab reduction beside the next kernel
                run_on_aux(dy.device, lambda: C.conv_wgrad(dy, inp, buf, s, p, d, 1.0, in_coef, fs), dy, inp, in_coef)
            else:
                C.conv_wgrad(dy, inp, buf, s, p, d, 1.0, in_coef)
            grad_done(w, direct)
            grads[id(w)] = None if direct else buf

        def dgrad(i, dy, shape, residual=None):
            s, p, d = _conv_conf(convs[i].conv)
            return C.conv_dgrad(dy, ws[i], shape, s, p, d, residual)

        def dgrad_bnb(i, dy, j, y, h, coef):
            """dL/dy of conv i's input, then BN j's backward.  With the fused epilogue the
            BN sums come out of the dgrad kernel and the ReLU mask is recomputed from h."""
            if not _EPI_BNB:
                da = dgrad(i, dy, list(h.shape))
                return bn_bwd(j, da, y, h, coef, False)[0]
            s, p, d = _conv_conf(convs[i].conv)
            da, part = C.conv_dgrad_bn(dy, ws[i], list(h.shape), s, p, d, None, h, coef)
            bn, gb, gd, bb, bd = bn_sinks(j)
            dh = C.bn_bwd_partials(da, h, bn.weight.detach(), coef, part, gb, bb)
            bn_done(bn, gb, gd, bb, bd)
            return dh

        lk = ctx.link_out
        chained = (lk is not None and lk.part is not None and lk.dz_ptr == dout.data_ptr()
                   and lk.dz_shape == tuple(dout.shape))
        gram = ctx.gram
        ctx.gram = None
        if gram is not None:
            # BN3 by Gram algebra: dz3 = dout came from the next block's epilogue with the sum-dz partials
            if not chained:
                raise RuntimeError("BN3 Gram path: the block output's gradient did not come from the chained epilogue")
            u3, sv, M3 = gram
            dz3 = dout
            src, src_coef = (h2, c2) if a2 is None else (a2, None)
            w3 = convs[2].conv.weight
            s3, p3, d3 = _conv_conf(convs[2].conv)
            P = torch.empty(w3.shape, dtype=torch.float32, device=w3.device)
            # P = dz3^T a2 with its K splits summed in a fixed order: BN3's dgamma comes from it (overwrite:
            # no zero fill of P)
            C.conv_wgrad(dz3, src, P, s3, p3, d3, 1.0, src_coef, deterministic=True, overwrite=True)
            bn, gb, gd, bb, bd = bn_sinks(2)
            wbuf, wdirect = grad_sink(w3)
            bcat, ebias = C.bn_gram_bwd(lk.part, P, ws[2], u3, sv, c3, bn.weight.detach(), M3, gb, bb, wbuf)
            bn_done(bn, gb, gd, bb, bd)
            grad_done(w3, wdirect)
            grads[id(w3)] = None if wdirect else wbuf
            dhd = None
            if has_down and lk.h3 is not None:  # BN_d's partials came with dz3 (forward: link_out.h3 = hd)
                bn, gb, gd, bb, bd = bn_sinks(3)
                dhd = C.bn_bwd_partials(dz3, hd, bn.weight.detach(), cd, lk.part, gb, bb, relu_mask=False)
                bn_done(bn, gb, gd, bb, bd)
            lk.part = None
            lk.h3 = lk.coef = lk.mask = None
            ctx.bits = None
            # da2 = [dz3 | a2] x [diag(a) W3 ; W3^T diag(b) W3] + c W3, with BN2's backward partials
            da2, part2 = C.conv1x1_dgrad_cat(dz3, src, src_coef, bcat, ebias, h2, c2)
            bn, gb, gd, bb, bd = bn_sinks(1)
            dh2 = C.bn_bwd_partials(da2, h2, bn.weight.detach(), c2, part2, gb, bb)
            bn_done(bn, gb, gd, bb, bd)
            return BottleneckFn._backward_tail(ctx, C, dz3, None, dh2, grads, bn_sinks, bn_done, bn_bwd, wgrad, dgrad,
                                               dgrad_bnb, dhd)
        if chained:
            # the next block's dgrad epilogue already produced dz3 = dout*relu'(out) and BN3's partials
            dz3 = dout
            bn, gb, gd, bb, bd = bn_sinks(2)
            if has_down and _BN_DUAL:
                # BN3 and the downsample BN both see dz3: one pass applies BN3's backward and
                # reduces BN_d's sums, then BN_d's apply (dz3 read twice instead of three times)
                bnd, gbd, gdd, bbd, bdd = bn_sinks(3)
                dh3, dhd = C.bn_bwd_dual(dz3, h3, bn.weight.detach(), c3, lk.part, gb, bb, hd, bnd.weight.detach(), cd,
                                         gbd, bbd)
                bn_done(bnd, gbd, gdd, bbd, bdd)
            elif _AX_BWD and _EPI_BNB and h3.shape[-1] <= _AX_BWD_MAXC and _ax_ok(convs[2].conv, h3.shape[-1]):
                # dh3 = a*dz3 + b*h3 + c computed on conv3's data-grad fragments (below), no apply pass
                dh3_coef = C.bn_bwd_coef(lk.part, h3.numel() // h3.shape[-1], bn.weight.detach(), c3, gb, bb)
            else:
                dh3 = C.bn_bwd_partials(dz3, h3, bn.weight.detach(), c3, lk.part, gb, bb, relu_mask=False)
            bn_done(bn, gb, gd, bb, bd)
            lk.part = None
        elif ctx.bits is not None and not has_down:
            # dz3 = dout * relu'(out) is only this block's residual gradient: the data-grad
            # epilogue masks dout with the bits itself, so dz3 is never written
            dh3, _ = bn_bwd(2, dout, out, h3, c3, False, ctx.bits)
            dz3, res_mask = dout, ctx.bits
        else:
            dh3, dz3 = bn_bwd(2, dout, out, h3, c3, True, ctx.bits)
        ctx.bits = None
        if lk is not None:
            lk.h3 = lk.coef = lk.mask = None
        if dh3_coef is not None:
            # conv3's data grad over dh3 = a*dz3 + b*h3 + c (on load), dh3 stored for the weight grad
            dh3 = torch.empty_like(h3)
            da2, part2 = C.conv1x1_bnin_dgrad(dz3, h3, dh3_coef, ws[2], dh3, h2, c2)
            bn, gb, gd, bb, bd = bn_sinks(1)
            dh2 = C.bn_bwd_partials(da2, h2, bn.weight.detach(), c2, part2, gb, bb)
            bn_done(bn, gb, gd, bb, bd)
            if a2 is None:
                wgrad(2, dh3, h2, c2)
            else:
                wgrad(2, dh3, a2)
        else:
            if a2 is None:  # a2 = relu(BN2(h2)) recomputed on the weight grad's B fragments
                wgrad(2, dh3, h2, c2)
            else:
                wgrad(2, dh3, a2)
            dh2 = dgrad_bnb(2, dh3, 1, a2, h2, c2)  # (a2 unused: _EPI_BNB recomputes the mask from h2)
        return BottleneckFn._backward_tail(ctx, C, dz3, res_mask, dh2, grads, bn_sinks, bn_done, bn_bwd, wgrad, dgrad,
                                           dgrad_bnb, dhd)

    @staticmethod
    def _backward_tail(ctx, C, dz3, res_mask, dh2, grads, bn_sinks, bn_done, bn_bwd, wgrad, dgrad, dgrad_bnb, dhd=None):
        """conv2 / conv1 / downsample gradients and dx, from dh2 (shared by the BN3 paths)."""
        x, h1, a1, h2, a2, h3, out, hd, c1, c2, c3, cd = ctx.saved_tensors
        convs, ws = ctx.convs, ctx.ws
        has_down = len(convs) == 4
        if a1 is None:  # a1 = relu(BN1(h1)) recomputed on load by the row-walking weight grad
            wgrad(1, dh2, h1, c1)
        else:
            wgrad(1, dh2, a1)
        dh1 = dgrad_bnb(1, dh2, 0, a1, h1, c1)  # (a1 unused: _EPI_BNB recomputes the mask from h1)
        wgrad(0, dh1, x)
        dx = None
        if ctx.needs_input_grad[0]:
            if has_down and ctx.link_in is not None:
                if dhd is None:
                    dhd, _ = bn_bwd(3, dz3, None, hd, cd, False)
                wgrad(3, dhd, x)
                li = ctx.link_in
                n, hh, ww, cin = x.shape
                dxd = C.conv_dgrad(dhd, ws[3], [n, hh // 2, ww // 2, cin], [1, 1], [0, 0], [1, 1])  # compact
                s, p, d = _conv_conf(convs[0].conv)
                if li.gram and li.h3 is None:  # the previous block's BN3 runs by Gram algebra: only the sum-dz partials
                    dx, part = C.conv_dgrad_bn(dh1, ws[0], list(x.shape), s, p, d, dxd, None, None, None, None, True,
                                               li.mask)
                else:
                    dx, part = C.conv_dgrad_bn(dh1, ws[0], list(x.shape), s, p, d, dxd, li.h3, li.coef, li.mask, None,
                                               True)
                li.part, li.dz_ptr, li.dz_shape = part, dx.data_ptr(), tuple(dx.shape)
            elif has_down:
                if dhd is None:
                    dhd, _ = bn_bwd(3, dz3, None, hd, cd, False)
                wgrad(3, dhd, x)
                dx = dgrad(0, dh1, list(x.shape))
                # downsample branch accumulated in place: a strided 1x1 only reaches one
                # output parity, the other three are never read or written
                s, p, d = _conv_conf(convs[3].conv)
                C.conv_dgrad_acc(dhd, ws[3], dx, s, p, d)
            elif ctx.link_in is not None:
                li = ctx.link_in
                s, p, d = _conv_conf(convs[0].conv)
                if li.gram and li.h3 is None:  # (li.h3 set: the previous block's downsample BN input, reduced too)
                    dx, part = C.conv_dgrad_bn(dh1, ws[0], list(x.shape), s, p, d, dz3, None, None, None, res_mask, False,
                                               li.mask)
                else:
                    dx, part = C.conv_dgrad_bn(dh1, ws[0], list(x.shape), s, p, d, dz3, li.h3, li.coef, li.mask, res_mask)
                li.part, li.dz_ptr, li.dz_shape = part, dx.data_ptr(), tuple(dx.shape)
            else:
                s, p, d = _conv_conf(convs[0].conv)
                dx = C.conv_dgrad(dh1, ws[0], list(x.shape), s, p, d, dz3, res_mask)
        elif has_down:
            if dhd is None:
                dhd, _ = bn_bwd(3, dz3, None, hd, cd, False)
            wgrad(3, dhd, x)
        pgrads = [grads.get(id(p)) for p in ctx.block._fused_params]
        return (dx, None, None, None, None, None, *pgrads)


def gram_successor_width(nxt) -> int:
    """For the block before ``nxt``: nxt's conv1 width when nxt will chain the BN3 backward in the form
    the Gram path needs (sum-dz partials from its conv1 data grad), else 0.  NEGATIVE for a downsample
    successor: the forward then also runs the successor's shape test (even H/W, strided-residual data
    grad on the streaming kernel) on the actual output shape before taking the Gram path."""
    if not _GRAM or nxt is None or not nxt.fused:
        return 0
    c1 = nxt.c1.conv
    if tuple(c1.kernel_size) != (1, 1) or tuple(c1.stride) != (1, 1):
        return 0
    if nxt.down is not None:
        d = nxt.down.conv
        if not (_DOWN_CHAIN and tuple(d.stride) == (2, 2) and tuple(d.kernel_size) == (1, 1)):
            return 0
        return -c1.out_channels
    return c1.out_channels


def bottleneck_forward(block, x, link_in=None, chain=False, count_batches=True, defer_out=False, gram_next=0):
    """Fused block forward.  ``chain=True`` (the ResNet's own block loop, where
    this block's output feeds only the next block) returns ``(out, link)`` for
    the next block's ``link_in``.  ``count_batches=False``: the ResNet advanced
    every block's num_batches_tracked in one launch already.  ``defer_out`` (with
    ``chain``; the next block passes ``can_materialise_input``): the returned
    output is written by the next block's conv1, which MUST be called next."""
    params = block._fused_params
    if count_batches:
        nbt = [cb.bn.num_batches_tracked
               for cb in [block.c1, block.c2, block.c3] + ([block.down] if block.down is not None else [])]
        torch._foreach_add_(nbt, 1)
    link_out = _BN3Link() if (chain and _BN3_CHAIN) else None
    out = BottleneckFn.apply(x, block, link_in if _BN3_CHAIN else None, link_out, bool(defer_out and link_out is not None),
                             int(gram_next) if link_out is not None else 0, *params)
    return (out, link_out) if chain else out
