"""Hand-scheduled forward/backward of a ResNet bottleneck block on gfx950.

One autograd node per block instead of ~12 per-op nodes:

forward  (x NHWC bf16)
    [hd = conv_d(x)  -> idn = BN_d(hd)]                          (downsample blocks)
    h1 = conv1(x)  -> a1 = relu(BN1(h1))      BN statistics come from the conv epilogue
    h2 = conv2(a1) -> a2 = relu(BN2(h2))
    h3 = conv3(a2) -> out = relu(BN3(h3) + idn)
backward (dout)
    dh3, dz3 = BN3'(dout; out, h3)            dz3 = dout*relu'(out) is also d(idn)
    dW3 += dh3 (x) a2 ;  da2 = dh3 . W3
    dh2 = BN2'(da2; a2, h2) ; dW2 += dh2 (x) a1 ; da1 = dh2 . W2
    dh1 = BN1'(da1; a1, h1) ; dW1 += dh1 (x) x
    identity block:   dx = dh1 . W1 + dz3            (residual add fused in the dgrad epilogue)
    downsample block: dhd = BN_d'(dz3; hd); dW_d += dhd (x) x
                      dx = dh1 . W1 + dhd . W_d      (second dgrad accumulates the first)

Weight gradients are accumulated straight into the DDP bucket views and each
parameter is announced to the reducer as soon as its gradient is final, in
reverse-forward order, so bucket all-reduces start while earlier blocks are
still in backward.
"""
from __future__ import annotations

import torch
from torch.autograd import Function

from ..ops._ext import ext
from ..ops._state import grad_done, grad_sink, note_use, shadow


def _conv_conf(conv):
    return list(conv.stride), list(conv.padding), list(conv.dilation)


class BottleneckFn(Function):
    @staticmethod
    def forward(ctx, x, block, *params):
        C = ext()
        convs = [block.c1, block.c2, block.c3] + ([block.down] if block.down is not None else [])
        ws = [shadow(cb.conv.weight) for cb in convs]
        coefs = []

        def convbn(i, inp, relu, residual=None):
            cb = convs[i]
            s, p, d = _conv_conf(cb.conv)
            h, st = C.conv_fwd(inp, ws[i], s, p, d, True, None)   # BN stats partials from the epilogue
            bn = cb.bn
            y, coef = C.bn_fwd_train(h, bn.weight.detach(), bn.bias.detach(), bn.running_mean, bn.running_var,
                                     bn.momentum, bn.eps, relu, residual, st)
            coefs.append(coef)
            return h, y

        if block.down is not None:
            hd, idn = convbn(3, x, False)
        else:
            hd, idn = None, x
        h1, a1 = convbn(0, x, True)
        h2, a2 = convbn(1, a1, True)
        h3, out = convbn(2, a2, True, idn)
        ctx.save_for_backward(x, h1, a1, h2, a2, h3, out, hd, *coefs)
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
        x, h1, a1, h2, a2, h3, out, hd, *coefs = ctx.saved_tensors
        convs, ws = ctx.convs, ctx.ws
        has_down = len(convs) == 4
        dout = dout.contiguous()

        def bn_bwd(i, dy, y, h, want_dz):
            bn = convs[i].bn
            gb, gd = grad_sink(bn.weight)
            bb, bd = grad_sink(bn.bias)
            dh, dz = C.bn_bwd(dy, y, h, bn.weight.detach(), coefs[i], gb, bb, want_dz)
            grad_done(bn.weight, gd)
            grad_done(bn.bias, bd)
            grads[id(bn.weight)] = None if gd else gb
            grads[id(bn.bias)] = None if bd else bb
            return dh, dz

        def wgrad(i, dy, inp):
            w = convs[i].conv.weight
            s, p, d = _conv_conf(convs[i].conv)
            buf, direct = grad_sink(w)
            C.conv_wgrad(dy, inp, buf, s, p, d, 1.0)
            grad_done(w, direct)
            grads[id(w)] = None if direct else buf

        def dgrad(i, dy, shape, residual=None):
            s, p, d = _conv_conf(convs[i].conv)
            return C.conv_dgrad(dy, ws[i], shape, s, p, d, residual)

        grads = {}
        # coefs are in forward order: [down], c1, c2, c3
        order = ([3] if has_down else []) + [0, 1, 2]
        coefs = {order[k]: coefs[k] for k in range(len(order))}

        dh3, dz3 = bn_bwd(2, dout, out, h3, True)
        wgrad(2, dh3, a2)
        da2 = dgrad(2, dh3, list(a2.shape))
        dh2, _ = bn_bwd(1, da2, a2, h2, False)
        wgrad(1, dh2, a1)
        da1 = dgrad(1, dh2, list(a1.shape))
        dh1, _ = bn_bwd(0, da1, a1, h1, False)
        wgrad(0, dh1, x)
        dx = None
        if ctx.needs_input_grad[0]:
            if has_down:
                dhd, _ = bn_bwd(3, dz3, None, hd, False)
                wgrad(3, dhd, x)
                dxd = dgrad(3, dhd, list(x.shape))
                dx = dgrad(0, dh1, list(x.shape), dxd)
            else:
                dx = dgrad(0, dh1, list(x.shape), dz3)
        elif has_down:
            dhd, _ = bn_bwd(3, dz3, None, hd, False)
            wgrad(3, dhd, x)
        pgrads = [grads.get(id(p)) for p in ctx.block._fused_params]
        return (dx, None, *pgrads)


def bottleneck_forward(block, x):
    params = block._fused_params
    nbt = [cb.bn.num_batches_tracked for cb in [block.c1, block.c2, block.c3] + ([block.down] if block.down is not None else [])]
    torch._foreach_add_(nbt, 1)
    return BottleneckFn.apply(x, block, *params)
