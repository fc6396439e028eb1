"""GPT-2 (BASELINE.json config 4: GPT-2-small, 124,439,808 parameters, T=1024).

Pre-LN transformer with tied token embedding / LM head, GELU(tanh) MLP, causal
self-attention, LayerNorm with bias -- the standard GPT-2 definition (same
parameterisation as HF/nanoGPT ``GPT2``), executed on gfx950 kernels:

* residual stream kept in fp32; LayerNorm reads it and emits bf16 for the GEMMs;
* QKV projection writes [B, T, 3, H, 64] which the flash-attention kernel reads
  in place (no split / transpose copies); attention output feeds the
  out-projection directly;
* the out-projections add into the fp32 residual stream inside the GEMM
  epilogue (one launch for ``x + proj(a)``);
* the LM head is the tied wte (bf16 shadow padded to a multiple of 64 rows),
  bf16 logits feed the fused cross-entropy kernel which writes bf16 dlogits.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import torch
import torch.nn as nn

from ..ops import functional as Fx
from ..ops.layers import LayerNorm, Linear

# DPE_GPT2_FUSED=0: per-op autograd graph for the blocks (A/B reference)
_FUSED = os.environ.get("DPE_GPT2_FUSED", "1") != "0"


@dataclass
class GPT2Config:
    vocab_size: int = 50257
    block_size: int = 1024
    n_layer: int = 12
    n_head: int = 12
    n_embd: int = 768
    dropout: float = 0.0
    bias: bool = True

    @classmethod
    def tiny(cls, **kw):
        base = dict(vocab_size=512, block_size=128, n_layer=2, n_head=2, n_embd=128)
        base.update(kw)
        return cls(**base)


class Block(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        d = cfg.n_embd
        self.n_head = cfg.n_head
        self.ln_1 = LayerNorm(d, bias=cfg.bias)
        self.c_attn = Linear(d, 3 * d, bias=cfg.bias)
        self.attn_proj = Linear(d, d, bias=cfg.bias)
        self.ln_2 = LayerNorm(d, bias=cfg.bias)
        self.c_fc = Linear(d, 4 * d, bias=cfg.bias)
        self.mlp_proj = Linear(4 * d, d, bias=cfg.bias)
        self.fused = _FUSED
        # every backward writes these through one weight-grad GEMM that honours grad_fresh (fused
        # and per-op paths alike): DDP may leave them out of the gradient re-zero (ops/_state.py)
        for lin in (self.c_attn, self.attn_proj, self.c_fc, self.mlp_proj):
            lin.weight._dpe_overwrite_ok = True

    def forward(self, x):
        if x.is_cuda and self.fused and torch.is_grad_enabled():
            from ._gpt2_fused import block_forward  # hand-scheduled fwd/bwd, one autograd node

            return block_forward(self, x)
        h = self.ln_1(x)
        qkv = self.c_attn(h)
        a = Fx.causal_attention(qkv, self.n_head)
        x = Fx.linear_residual(a, self.attn_proj.weight, self.attn_proj.bias, x)
        h = self.ln_2(x)
        u = Fx.gelu(self.c_fc(h))
        return Fx.linear_residual(u, self.mlp_proj.weight, self.mlp_proj.bias, x)


class GPT2(nn.Module):
    def __init__(self, cfg: GPT2Config = GPT2Config()):
        super().__init__()
        self.cfg = cfg
        self.wte = nn.Parameter(torch.empty(cfg.vocab_size, cfg.n_embd))
        self.wpe = nn.Parameter(torch.empty(cfg.block_size, cfg.n_embd))
        self.h = nn.ModuleList([Block(cfg) for _ in range(cfg.n_layer)])
        for i, blk in enumerate(self.h):
            blk._dpe_layer = i  # the fused backward flushes deferred weight grads at layer 0 (end of backward)
        self.ln_f = LayerNorm(cfg.n_embd, bias=cfg.bias)
        # tied LM head / embedding: the LM-head weight grad (first writer) overwrites when fresh, the
        # embedding scatter-add accumulates after it
        self.wte._dpe_overwrite_ok = True
        self._init()

    def _init(self):
        # GPT-2 init: N(0, 0.02); residual projections scaled by 1/sqrt(2*n_layer)
        std = 0.02
        with torch.no_grad():
            self.wte.normal_(0, std)
            self.wpe.normal_(0, std)
            for blk in self.h:
                for lin in (blk.c_attn, blk.c_fc):
                    lin.weight.normal_(0, std)
                    if lin.bias is not None:
                        lin.bias.zero_()
                for lin in (blk.attn_proj, blk.mlp_proj):
                    lin.weight.normal_(0, std / math.sqrt(2 * self.cfg.n_layer))
                    if lin.bias is not None:
                        lin.bias.zero_()

    def forward(self, idx, targets=None):
        """Logits [B, T, V(p)], or -- with ``targets`` -- the mean next-token
        cross-entropy through the fused LM-head + CE op (logits never materialise
        outside it)."""
        B, T = idx.shape
        assert T <= self.cfg.block_size, "sequence longer than block_size"
        if _FUSED and idx.is_cuda:
            from ._gpt2_fused import reset_wgrad_queue

            reset_wgrad_queue()
        x = Fx.embedding(idx, self.wte, self.wpe[:T] if not idx.is_cuda else self.wpe)
        for blk in self.h:
            x = blk(x)
        x = self.ln_f(x)
        if targets is not None:
            return Fx.lm_head_ce(x, self.wte, targets)
        return Fx.lm_head(x, self.wte)

    def num_params(self) -> int:
        return sum(p.numel() for p in self.parameters())
