"""Hand-scheduled forward/backward of a GPT-2 pre-LN transformer block on gfx950.

One autograd node per block instead of eight per-op nodes.  The per-op graph
pays, per block, two fp32->bf16 casts of the residual-stream gradient and two
fp32 adds where autograd joins the residual branch with the LayerNorm branch;
here both disappear into the LayerNorm backward kernel (residual form: it reads
the incoming stream gradient, adds the LN input gradient and writes the result
in fp32 *and* bf16 in one pass):

forward  (x fp32 residual stream [B, T, D])
    h1 = LN1(x)                     bf16
    qkv = h1 W_qkv^T + b            bf16 [B, T, 3, H, 64], read in place by attention
    a, lse = attn(qkv)              causal flash attention
    x2 = x + a W_o^T + b            fp32, residual add in the GEMM epilogue
    h2 = LN2(x2) ; v = h2 W_fc^T + b ; u = gelu(v)   one GEMM: u and v from its epilogue
    y  = x2 + u W_p^T + b           fp32
backward (g = dL/dy fp32, gb its bf16 copy)
    dW_p += gb^T u , db_p += colsum(gb) (one launch) ; dv = gelu'(v) (gb W_p)   (GELU' in the GEMM epilogue)
    dW_fc += dv^T h2 ; db_fc ; dh2 = dv W_fc
    g2, g2b = g + LN2'(dh2)         one kernel: fp32 stream grad + bf16 copy
    dW_o += g2b^T a ; db_o ; da = g2b W_o ; dqkv = attn'(da)
    dW_qkv += dqkv^T h1 ; db_qkv ; dh1 = dqkv W_qkv
    g1, g1b = g2 + LN1'(dh1)        -> returned; g1b handed to the previous block

The bf16 copy of the returned gradient is passed to the next backward node
(the previous block) through ``_carry``: it is used only if that node receives
exactly the tensor this node returned (same storage, shape and version), else
the node casts itself.  Weight gradients go straight into the DDP bucket views
and are announced in reverse-forward order, as in the per-op path.

Reference parity: the reference trains only SimpleNet (``train.py``); GPT-2 is
BASELINE.json config 4 -- same math as ``models/gpt2.py:Block``.
"""
from __future__ import annotations

import math
import os

import torch
from torch.autograd import Function

from ..ops._ext import ext
from ..ops._state import finalize_stream, grad_done, grad_fresh, grad_sink, note_use, shadow

# (fp32 grad, its bf16 copy, version) produced by the most recent block backward
_carry: list = [None]

# Grouped weight gradients.  Alone, a layer's four weight-grad GEMMs (dW = dy^T x over K = B*T tokens;
# 27 / 9 / 36 / 36 output tiles of 256x256 at d = 768) need an 8-9-way K split each to fill 256 CUs,
# and the split's fp32 partial slabs plus their finalize launch cost about as much as the GEMM itself.
# Deferred here and launched together (C.linear_wgrad_group, hgemm HE_GROUP: whole-K tiles, no slabs) in
# whole rounds of the persistent grid (below; DPE_GPT2_WGRAD_GROUP=0: no grouping).  Only gradients
# that live in DDP bucket views are deferred (the reducer is told when the group has been written; a
# gradient autograd would receive from this node must be complete when backward returns).  0 = off.
_WG_GROUP = int(os.environ.get("DPE_GPT2_WGRAD_GROUP", "2"))
# Launches are cut by output tiles, not by layers: a grouped launch takes the longest queue prefix of at most
# one round of 256x256 tiles (the persistent grid: CUs minus the RCCL-reserved slots, _wg_round) and
# HGEMM_MAX_GROUP problems; what does not fill a round
# waits for the next layer, and at the end of backward a remainder under half a round runs as ordinary
# (K-split) weight-grad GEMMs instead of a mostly idle round.  GPT-2-small: 1296 tiles -> 5 launches of
# 252 + 36 tiles alone (was 6 launches of 216).  DPE_GPT2_WGRAD_POLICY=layers: the _WG_GROUP-layer groups (A/B).
_WG_TILES_ENV = os.environ.get("DPE_GPT2_WGRAD_TILES")


def _wg_round(C) -> int:
    """Tiles of one round of the grouped launch's persistent grid right now: the device's CUs minus the
    slots left to resident RCCL blocks (the CU budget, while a bucket all-reduce is in flight) -- the grid
    linear_wgrad_group launches, so a round-sized group never spills into a second round."""
    if _WG_TILES_ENV:
        return int(_WG_TILES_ENV)
    return max(64, C.num_cus() - C.cu_reserve())
_WG_BY_TILES = os.environ.get("DPE_GPT2_WGRAD_POLICY", "tiles") != "layers"
_wq: list = []  # (dy, x, dw, db | None, overwrite, weight param, bias param | None)
# The LayerNorm weight / bias gradients of the same layers: their [blocks][2][D] partial sums are kept and
# reduced by one grouped launch at the same flush (a standalone finalize is a ~5 us latency-bound launch,
# two per block).  DPE_GPT2_LN_GROUP=0: finalized per LayerNorm.
_LN_GROUP = os.environ.get("DPE_GPT2_LN_GROUP", "1") == "1"
_lnq: list = []  # (part, rows, dw, db | None, weight param, bias param | None)


def reset_wgrad_queue() -> None:
    """Drop deferred work of a backward that raised (called at every forward)."""
    for q in _wq:
        q[5]._dpe_deferred = False
        if q[6] is not None:
            q[6]._dpe_deferred = False
    _wq.clear()
    for q in _lnq:
        q[4]._dpe_deferred = False
        if q[5] is not None:
            q[5]._dpe_deferred = False
    _lnq.clear()


def flush_ln_queue() -> None:
    """Reduce the queued LayerNorm weight / bias partials (groups of at most 8) and announce them."""
    if not _lnq:
        return
    C = ext()
    items = list(_lnq)
    _lnq.clear()
    for i in range(0, len(items), 8):
        chunk = items[i:i + 8]
        C.layernorm_bwd_finalize_group([q[0] for q in chunk], [q[1] for q in chunk], [q[2] for q in chunk],
                                       [q[3] for q in chunk])
    for q in items:
        q[4]._dpe_deferred = False
        if q[5] is not None:
            q[5]._dpe_deferred = False
    for q in items:
        grad_done(q[4], True)
        if q[5] is not None:
            grad_done(q[5], True)


def _wg_tiles(q) -> int:
    M, N = q[2].shape[0], q[2].shape[1]
    return ((M + 255) // 256) * ((N + 255) // 256)


def _wg_launch_group(C, chunk) -> None:
    C.linear_wgrad_group([q[0] for q in chunk], [q[1] for q in chunk], [q[2] for q in chunk],
                         [q[3] if q[3] is not None else _EMPTY(q[2]) for q in chunk], [q[4] for q in chunk])


def flush_wgrad_queue(final: bool = True) -> None:
    """Launch queued weight gradients and announce them.  ``final`` (end of backward, a token-count change, or
    grouping off): everything; else (tile policy) only the whole-round prefixes, the rest stays queued."""
    flush_ln_queue()
    if not _wq:
        return
    C = ext()
    items = []
    if not _WG_BY_TILES:
        items = list(_wq)
        _wq.clear()
        for i in range(0, len(items), 8):
            _wg_launch_group(C, items[i:i + 8])
    else:
        rnd, maxp = _wg_round(C), C.HGEMM_MAX_GROUP
        while _wq:
            n, t = 0, 0
            while n < len(_wq) and n < maxp and t + _wg_tiles(_wq[n]) <= rnd:
                t += _wg_tiles(_wq[n])
                n += 1
            n = max(n, 1)  # (a problem of more than one round alone)
            if n == len(_wq) and not final:
                break  # the queue fits in one round: wait for the next layer's problems
            chunk = _wq[:n]
            del _wq[:n]
            if n == len(chunk) and not _wq and final and t < rnd // 2:
                for q in chunk:  # a small remainder: ordinary K-split GEMMs (planner) instead of an idle round
                    C.linear_wgrad(q[0], q[1], q[2], 1.0, None, q[3], 0, q[4])
            else:
                _wg_launch_group(C, chunk)
            items += chunk
    for q in items:
        q[5]._dpe_deferred = False
        if q[6] is not None:
            q[6]._dpe_deferred = False
    for q in items:
        grad_done(q[5], True)
        if q[6] is not None:
            grad_done(q[6], True)


def _EMPTY(like):
    return like.new_empty(0)


def _bf16_of(g: torch.Tensor) -> torch.Tensor:
    c = _carry[0]
    _carry[0] = None
    if c is not None:
        g32, gb, ver = c
        if (g32.data_ptr() == g.data_ptr() and g32.shape == g.shape and g.dtype == torch.float32
                and g._version == ver and g.is_contiguous()):
            return gb
    return g.to(torch.bfloat16).contiguous()


def block_params(blk):
    """Parameters of ``blk`` in the order BlockFn takes them (None biases skipped)."""
    mods = (blk.ln_1, blk.c_attn, blk.attn_proj, blk.ln_2, blk.c_fc, blk.mlp_proj)
    return [t for m in mods for t in (m.weight, m.bias) if t is not None]


class BlockFn(Function):
    @staticmethod
    def forward(ctx, x, blk, *params):
        C = ext()
        B, T, D = x.shape
        H = blk.n_head
        hd = D // H
        scale = 1.0 / math.sqrt(hd)
        x = x.contiguous()

        def opt(t):
            return t.detach() if t is not None else None

        h1, m1, r1 = C.layernorm_fwd(x, blk.ln_1.weight.detach(), opt(blk.ln_1.bias), blk.ln_1.eps)
        qkv = C.linear_fwd(h1, shadow(blk.c_attn.weight), opt(blk.c_attn.bias), 0, False, None, None)
        qkv5 = qkv.view(B, T, 3, H, hd)
        a, lse = C.attn_fwd(qkv5, H, scale, True)
        a = a.view(B, T, D)
        x2 = C.linear_fwd(a, shadow(blk.attn_proj.weight), opt(blk.attn_proj.bias), 0, True, x, None)
        h2, m2, r2 = C.layernorm_fwd(x2, blk.ln_2.weight.detach(), opt(blk.ln_2.bias), blk.ln_2.eps)
        # GELU in the GEMM epilogue; the pre-activation v is written alongside for the backward
        v = torch.empty((B, T, blk.c_fc.weight.shape[0]), device=x.device, dtype=torch.bfloat16)
        u = C.linear_fwd(h2, shadow(blk.c_fc.weight), opt(blk.c_fc.bias), 2, False, None, None, v)
        y = C.linear_fwd(u, shadow(blk.mlp_proj.weight), opt(blk.mlp_proj.bias), 0, True, x2, None)
        ctx.save_for_backward(x, h1, m1, r1, qkv5, a, lse, x2, h2, m2, r2, v, u)
        ctx.blk, ctx.scale = blk, scale
        for p in params:
            note_use(p)
        return y

    @staticmethod
    def backward(ctx, g):
        C = ext()
        x, h1, m1, r1, qkv5, a, lse, x2, h2, m2, r2, v, u = ctx.saved_tensors
        blk = ctx.blk
        g = g.contiguous()
        gb = _bf16_of(g)
        grads = {}
        T = g.numel() // g.shape[-1]
        group = _WG_GROUP > 0 and T % 64 == 0 and g.shape[-1] % 8 == 0

        def sink(p):
            buf, direct = grad_sink(p)
            return buf, direct

        def done(p, buf, direct):
            grad_done(p, direct)
            grads[id(p)] = None if direct else buf

        def linear_bwd(lin, dyb, inp, want_dx=True, gelu_in=None):
            """dW += dyb^T inp and db += colsum(dyb) in one GEMM launch ; return dyb W (bf16), times gelu'(gelu_in) if given."""
            buf, d = sink(lin.weight)
            bb, bd = sink(lin.bias) if lin.bias is not None else (None, True)
            if group and d and bd:
                # deferred to the grouped launch at the end of this block's (or the next one's) backward;
                # DDP's post-accumulate hook (which fires after this node returns) must not announce them
                lin.weight._dpe_deferred = True
                if lin.bias is not None:
                    lin.bias._dpe_deferred = True
                _wq.append((dyb, inp, buf, bb, grad_fresh(lin.weight), lin.weight, lin.bias))
                return C.linear_dgrad(dyb, shadow(lin.weight), None, None, gelu_in) if want_dx else None
            # bias grad from the same launch (row sums of dy^T); a K-split's slab reduction may run on the
            # side stream when both gradients are bucket views (the reducer / backward join wait for it)
            fs = finalize_stream(dyb.device) if (d and bd) else 0
            C.linear_wgrad(dyb, inp, buf, 1.0, None, bb, fs, d and grad_fresh(lin.weight))
            done(lin.weight, buf, d)
            if lin.bias is not None:
                done(lin.bias, bb, bd)
            return C.linear_dgrad(dyb, shadow(lin.weight), None, None, gelu_in) if want_dx else None

        def ln_bwd(ln, dy, xin, mean, rstd, res):
            wb, wd = sink(ln.weight)
            bb, bd = sink(ln.bias) if ln.bias is not None else (None, False)
            if group and _LN_GROUP and wd and (ln.bias is None or bd):
                # partials kept; reduced into the bucket views by the grouped launch at the next flush
                ln.weight._dpe_deferred = True
                if ln.bias is not None:
                    ln.bias._dpe_deferred = True
                dx, dxb, part = C.layernorm_bwd_residual(dy, xin, ln.weight.detach(), mean, rstd, wb, bb, res, True)
                _lnq.append((part, xin.numel() // xin.shape[-1], wb, bb, ln.weight, ln.bias))
                grads[id(ln.weight)] = None
                if ln.bias is not None:
                    grads[id(ln.bias)] = None
                return dx, dxb
            dx, dxb = C.layernorm_bwd_residual(dy, xin, ln.weight.detach(), mean, rstd, wb, bb, res)
            done(ln.weight, wb, wd)
            if ln.bias is not None:
                done(ln.bias, bb, bd)
            return dx, dxb

        # one grouped launch needs one token count: a backward over two graphs of different B*T (two
        # micro-batches' losses summed) flushes what the other graph queued before queueing its own
        if (_wq and _wq[0][0].numel() // _wq[0][0].shape[-1] != T) or (_lnq and _lnq[0][1] != T):
            flush_wgrad_queue()
        dv = linear_bwd(blk.mlp_proj, gb, u, gelu_in=v)  # GELU backward in the data-grad epilogue
        dh2 = linear_bwd(blk.c_fc, dv, h2)
        g2, g2b = ln_bwd(blk.ln_2, dh2, x2, m2, r2, g)
        da = linear_bwd(blk.attn_proj, g2b, a)
        dqkv = C.attn_bwd(qkv5, a.view(qkv5.shape[0], qkv5.shape[1], qkv5.shape[3], qkv5.shape[4]), da, lse,
                          blk.n_head, ctx.scale, True)
        dqkv = dqkv.view(a.shape[0], a.shape[1], -1)
        dh1 = linear_bwd(blk.c_attn, dqkv, h1)
        g1, g1b = ln_bwd(blk.ln_1, dh1, x, m1, r1, g2)
        last = getattr(blk, "_dpe_layer", 0) == 0 or not group
        if _WG_BY_TILES:
            if (_wq or _lnq) and (last or sum(_wg_tiles(q) for q in _wq) > _wg_round(ext())):
                flush_wgrad_queue(final=last)  # whole rounds as they fill, everything at the first block
        elif (_wq or _lnq) and (len(_wq) >= 4 * _WG_GROUP or last):
            flush_wgrad_queue()  # every _WG_GROUP layers, and always at the first block (end of backward)
        _carry[0] = (g1, g1b, g1._version)
        pgrads = [grads.get(id(p)) for p in block_params(blk)]
        return (g1, None, *pgrads)


def block_forward(blk, x):
    return BlockFn.apply(x, blk, *block_params(blk))

