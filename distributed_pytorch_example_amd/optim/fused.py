"""Fused multi-tensor optimizers (Adam / AdamW / SGD-momentum).

Drop-in subclasses of the torch optimizers: identical constructor arguments,
identical ``state_dict()`` schema (so checkpoints interchange with the
reference's ``optim.Adam``), identical update math.  On GPU the
whole step is ONE HIP kernel launch over a device-resident (tensor, chunk)
table (csrc/kernels/optim.hip) that also refreshes each parameter's bf16
compute shadow; on CPU they defer to torch's implementation.

Replaces the reference's foreach-Adam (`train.py:249` ->
`$TORCH/optim/adam.py:554` `_multi_tensor_adam`: lerp/mul/addcmul/sqrt/div/
add/addcdiv launches per step).

Per-parameter ``step`` counters live in one device tensor (each state's
``step`` is a 0-d view of it), so a whole training step can be captured in a
hipGraph; ``lr`` and friends live in a device hyper-parameter block that the
host rewrites only when a group's values change.
"""
from __future__ import annotations

import struct

import torch

from ..ops._ext import ext
from ..ops import _state

_HP = 12


class _FusedMixin:
    _kind = 0  # 0 adam, 1 sgd

    def _fused_init(self):
        self._tab = None
        self._tab_key = None
        self._hp_key = None
        self._hp = None
        self._steps = None
        self.graph_safe = False  # when True: skip per-step host checks (caller guarantees static pointers)
        self._ov_stream = None  # DDP.overlap_optimizer: per-bucket steps during backward on this stream
        self._ov_open = False
        self._ov_done = set()
        self._ov_cache = {}

    def _all_params(self):
        return [p for g in self.param_groups for p in g["params"]]

    def _use_fused(self) -> bool:
        ps = self._all_params()
        return len(ps) > 0 and all(p.is_cuda for p in ps)

    # -------------------------------------------------------- state setup
    def _ensure_state(self):
        params = self._all_params()
        dev = params[0].device
        if self._steps is None or self._steps.numel() != len(params):
            steps = torch.zeros(len(params), dtype=torch.float32, device=dev)
            for i, p in enumerate(params):
                st = self.state.get(p)
                if st and "step" in st:
                    steps[i] = float(st["step"])
                elif st and st.get("momentum_buffer") is not None:
                    # a stock torch.optim.SGD state has a momentum buffer but no step counter: the kernel's
                    # "first step" (b = g) must not discard the loaded buffer
                    steps[i] = 1.0
            self._steps = steps
        for i, p in enumerate(params):
            st = self.state[p]
            if self._kind == 0:
                if "exp_avg" not in st:
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            else:
                g = self._group_of(p)
                if g["momentum"] != 0 and st.get("momentum_buffer") is None:
                    st["momentum_buffer"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            if st.get("step") is None or st["step"].data_ptr() != self._steps[i].data_ptr():
                st["step"] = self._steps[i]

    def _group_of(self, p):
        for g in self.param_groups:
            for q in g["params"]:
                if q is p:
                    return g
        raise KeyError

    def _build_table(self):
        C = ext()
        chunk = C.optim_chunk_size()
        params = self._all_params()
        desc = bytearray()
        chunks = []
        self._ti = {}
        gi_of = {}
        for gi, g in enumerate(self.param_groups):
            for p in g["params"]:
                gi_of[id(p)] = gi
        for ti, p in enumerate(params):
            st = self.state[p]
            if p.grad is None:
                raise RuntimeError("fused optimizer: parameter without .grad (use zero_grad(set_to_none=False) or DDP)")
            if not (p.is_contiguous() and p.grad.is_contiguous()):
                raise RuntimeError("fused optimizer needs contiguous params/grads")
            s1 = st["exp_avg"] if self._kind == 0 else st.get("momentum_buffer")
            s2 = st["exp_avg_sq"] if self._kind == 0 else None
            sh = getattr(p, "_dpe_shadow", None)
            if sh is not None and getattr(p, "_dpe_shadow_ver", -1) != p._version:
                sh = None  # stale shadow: let the layer re-cast it
            self._ti[id(p)] = ti
            desc += struct.pack("<QQQQQqii", p.data_ptr(), p.grad.data_ptr(), s1.data_ptr() if s1 is not None else 0,
                                s2.data_ptr() if s2 is not None else 0, sh.data_ptr() if sh is not None else 0,
                                p.numel(), gi_of[id(p)], ti)
            for c in range((p.numel() + chunk - 1) // chunk):
                chunks.append((ti, c))
        assert len(desc) == C.optim_desc_bytes() * len(params), "TensorDesc ABI mismatch"
        dev = params[0].device
        d = torch.frombuffer(desc, dtype=torch.uint8).to(dev)
        ck = torch.tensor(chunks, dtype=torch.int32).reshape(-1, 2).to(dev)
        self._tab = (d, ck)
        self._chunks_host = chunks
        self._ov_cache = {}

    def _key(self):
        ks = []
        for p in self._all_params():
            st = self.state[p]
            sh = getattr(p, "_dpe_shadow", None)
            s1 = st.get("exp_avg") if self._kind == 0 else st.get("momentum_buffer")
            s2 = st.get("exp_avg_sq") if self._kind == 0 else None
            ks.append((p.data_ptr(), p.grad.data_ptr() if p.grad is not None else 0,
                       sh.data_ptr() if sh is not None and getattr(p, "_dpe_shadow_ver", -1) == p._version else 0,
                       s1.data_ptr() if s1 is not None else 0, s2.data_ptr() if s2 is not None else 0))
        return tuple(ks)

    def load_state_dict(self, state_dict):
        """torch's load puts fresh state tensors in ``self.state`` (the old ones go back to the caching
        allocator): drop the device table and the step counters so the next fused step rebuilds both
        from the loaded state instead of touching freed memory."""
        super().load_state_dict(state_dict)
        self._steps = None
        self._tab = None
        self._tab_key = None
        self._hp_key = None

    def _hp_row(self, g):
        raise NotImplementedError

    def _write_hp(self):
        rows = [self._hp_row(g) for g in self.param_groups]
        key = tuple(tuple(r) for r in rows)
        if key != self._hp_key:
            t = torch.tensor([v for r in rows for v in r], dtype=torch.float32)
            if self._hp is None or self._hp.numel() != t.numel():
                self._hp = t.to(self._all_params()[0].device)
            else:
                self._hp.copy_(t, non_blocking=False)
            self._hp_key = key

    # -------------------------------------------- optimizer in backward (DDP.overlap_optimizer)
    def _ov_attach(self, stream):
        self._ov_stream, self._ov_open, self._ov_done = stream, False, set()

    def _ov_detach(self):
        if self._ov_open:
            # buckets of this iteration were already stepped during backward: detaching now would leave
            # the rest for a normal step() that re-steps everything (a silent double update)
            raise RuntimeError("overlap_optimizer(enable=False) between backward and optimizer.step(): "
                               "call optimizer.step() first to finish the iteration's overlapped update")
        self._ov_stream, self._ov_open = None, False

    def _ov_launch(self, tis, stream):
        """The fused kernel over the chunks of tensors ``tis`` only (chunk lists cached per bucket)."""
        key = tuple(tis)
        ck = self._ov_cache.get(key)
        if ck is None:
            want = set(key)
            ck = torch.tensor([c for c in self._chunks_host if c[0] in want], dtype=torch.int32).reshape(-1, 2).to(
                self._tab[0].device)
            self._ov_cache[key] = ck
        with torch.cuda.stream(stream):
            ext().optim_step(self._kind, self._tab[0], ck, self._hp, self._steps)
        self._ov_done.update(key)

    @torch.no_grad()
    def _ov_bucket_step(self, params, stream):
        """Step ``params`` (one DDP bucket whose gradients are final and whose readers have returned) on
        ``stream``, which the caller has already ordered after them.  The first bucket of an iteration
        refreshes the device table / hyper-parameters and advances every step counter once."""
        if not self._ov_open:
            with torch.cuda.stream(stream):
                self._ensure_state()
                key = self._key()
                if key != self._tab_key:
                    self._build_table()
                    self._tab_key = key
                self._write_hp()
                self._steps.add_(1.0)
            self._ov_open, self._ov_done = True, set()
        tis = sorted({self._ti[id(p)] for p in params if id(p) in self._ti} - self._ov_done)
        if tis:
            self._ov_launch(tis, stream)

    @torch.no_grad()
    def _fused_step(self):
        if self._ov_open:
            # the buckets were stepped during backward: step anything left, then join the stream
            rest = [ti for ti in range(len(self._all_params())) if ti not in self._ov_done]
            if rest:
                self._ov_launch(rest, self._ov_stream)
            torch.cuda.current_stream().wait_stream(self._ov_stream)
            self._ov_open = False
            _state.after_optimizer_step()
            return
        if not self.graph_safe or self._tab is None:
            self._ensure_state()
            key = self._key()
            if key != self._tab_key:
                self._build_table()
                self._tab_key = key
            self._write_hp()
        self._steps.add_(1.0)
        d, ck = self._tab
        ext().optim_step(self._kind, d, ck, self._hp, self._steps)
        _state.after_optimizer_step()


def _lr(g):
    lr = g["lr"]
    return float(lr.item() if torch.is_tensor(lr) else lr)


class Adam(_FusedMixin, torch.optim.Adam):
    """torch.optim.Adam with a one-launch fused HIP step on GPU."""

    _kind = 0
    _decoupled = False

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False, *,
                 maximize=False, **kw):
        if amsgrad:
            raise NotImplementedError("amsgrad is not supported by the fused kernel")
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False,
                         maximize=maximize, **kw)
        self._fused_init()

    def _hp_row(self, g):
        flags = (2 if g.get("maximize", False) else 0) | (4 if (self._decoupled or g.get("decoupled_weight_decay", False)) else 0)
        b1, b2 = g["betas"]
        return [_lr(g), float(b1), float(b2), float(g["eps"]), float(g["weight_decay"]), float(flags), 1.0] + [0.0] * (_HP - 7)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self._use_fused():
            self._fused_step()
            return loss
        return super().step()


class AdamW(Adam):
    _decoupled = True

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, amsgrad=False, **kw):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad,
                         decoupled_weight_decay=True, **kw)


class SGD(_FusedMixin, torch.optim.SGD):
    """torch.optim.SGD (momentum / nesterov / weight decay) with a fused HIP step on GPU."""

    _kind = 1

    def __init__(self, params, lr=1e-3, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False, *,
                 maximize=False, **kw):
        super().__init__(params, lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                         nesterov=nesterov, maximize=maximize, **kw)
        self._fused_init()

    def _hp_row(self, g):
        flags = (1 if g["nesterov"] else 0) | (2 if g.get("maximize", False) else 0)
        return [_lr(g), float(g["momentum"]), float(g["dampening"]), 0.0, float(g["weight_decay"]), float(flags), 1.0] + [
            0.0] * (_HP - 7)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self._use_fused():
            self._fused_step()
            return loss
        return super().step()
