"""DistributedDataParallel for MI355X.

API-compatible subset of ``torch.nn.parallel.DistributedDataParallel`` as the
reference uses it (`train.py:12,233`: ``DDP(model)``, ``.module``, forward,
implicit gradient averaging in backward) plus ``no_sync()``,
``broadcast_buffers``, bucket-size control, ``register_comm_hook`` and the
one-time bucket rebuild from the observed gradient-ready order (SURVEY §2.2
I4/I5).

Design (MI355X-first, not a port of c10d::Reducer):

* **Flat buckets, gradient-as-bucket-view.**  Every parameter's ``.grad`` is
  a view into a flat fp32 bucket buffer for the whole run.  Our backward
  kernels (Linear/Conv/BN/LN/Embedding) atomically accumulate weight
  gradients *directly* into that view and announce readiness themselves --
  there is no grad->bucket copy-and-scale (c10d's ``mul_out``, K18) and no
  bucket->grad copy-back (K20).  Parameters of foreign modules still work via
  ``register_post_accumulate_grad_hook``.
* **Native reducer.**  On the rccl backend the per-bucket all-reduce is
  issued by the C++ ``_C.Reducer`` on the communicator's high-priority side
  stream behind an event recorded on the compute stream, so RCCL overlaps the
  rest of backward; averaging uses ``ncclAvg`` (no scale kernel).  Buckets are
  issued strictly in index order on every rank.  At the end of backward the
  compute stream waits for the last bucket.  ``gradient_compression="bf16"``
  (or ``register_comm_hook(None, bf16_compress_hook)``) all-reduces bf16
  copies cast on the comm stream.
* **Bucket rebuild.**  Like c10d (`distributed.py:1201-1206`), the buckets
  are rebuilt once, before the second forward, in the order gradients were
  observed to become ready in the first backward -- rank 0's order is
  broadcast so every rank builds identical buckets.
* **Desync guard.**  ``debug=True`` (or ``DPE_DDP_DEBUG=1``) fingerprints the
  bucket layout at every (re)build and compares it across ranks through the
  control plane (fail fast instead of hanging in mismatched collectives), and
  synchronises the comm stream after every bucket.
* **gloo / CPU**: the same C++ reducer in host-transport mode (readiness,
  index-order issue and finalize in C++; the bucket all-reduce delegated to
  gloo).  Custom comm hooks run on a Python reducer.
* **Init sync**: parameters and buffers are broadcast from rank 0 as one flat
  buffer per dtype (c10d's coalesced broadcast, C3).
* **Buffer sync (C9)**: with ``broadcast_buffers`` the module's buffers
  (BatchNorm running stats: 53,120 floats for ResNet-50, plus the 53 int64
  ``num_batches_tracked`` counters) are re-homed
  once as views of ONE flat tensor per dtype/device, so the per-forward
  broadcast is a single RCCL call with no concatenate / scatter-back copies
  (c10d coalesces into a temporary and copies back: ~2 tiny kernels per
  buffer per step).
* **Optimizer in backward** (``overlap_optimizer(opt)``, opt-in): the fused optimizer's step runs per
  gradient bucket on its own stream DURING backward -- bucket b is stepped once its gradients are final
  (and, at world > 1, all-reduced) and every autograd node that read its parameters has returned (their
  post-accumulate hooks fired), so no backward kernel can read a weight the step rewrites.  The
  memory-bound update overlaps the compute-bound tail of backward instead of following it; ``opt.step()``
  then only joins the stream (and steps anything left).  Same math, same order per parameter.
"""
from __future__ import annotations

import contextlib
import hashlib
import os
import time
from typing import Callable, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from . import dist as pdist
from . import hooks as _hooks
from ..ops import _state
from .buckets import assign_buckets, xgmi_bucket_policy
from ..utils.logging import get_logger
from ..ops._state import aux_wait as _aux_wait

log = get_logger(__name__)


def _has_ext() -> bool:
    from ..ops._ext import has_ext

    return has_ext()

_DEFAULT_FIRST_BUCKET_BYTES = 1024 * 1024



# DPE_GRAD_FRESH=0: re-zero every gradient bucket (A/B arm of the overwrite-first-write protocol)
_GRAD_FRESH = os.environ.get("DPE_GRAD_FRESH", "1") != "0"

class _PyReducer:
    """Python reducer: gloo backend, or any backend with a user comm hook.

    Buckets are handed to the hook (default: async all-reduce + average) in
    index order as they complete; ``finalize`` waits for all of them."""

    def __init__(self, buckets: List[torch.Tensor], bucket_params: List[List[int]], nparams: int, params,
                 hook: Optional[Callable] = None, state=None, compression: Optional[str] = None):
        self.buckets = buckets
        self.bucket_params = bucket_params
        self.params = params
        self.bucket_of = {}
        for b, ps in enumerate(bucket_params):
            for p in ps:
                self.bucket_of[p] = b
        self.expected = [len(ps) for ps in bucket_params]
        self.world = pdist.get_world_size()
        self.hook, self.state, self.compression = hook, state, compression
        self.order: List[int] = []
        self.prepare()

    def prepare(self):
        self.pending = list(self.expected)
        self.ready = [False] * len(self.buckets)
        self.seen = set()
        self.next = 0
        self.works = []
        self.open = True
        self.order = []

    def _launch(self, b):
        self.order.append(b)
        t = self.buckets[b]
        if t.is_cuda:
            _aux_wait(t.device)  # weight grads written on the side stream
        if self.hook is not None:
            gb = _hooks.GradBucket(b, t, [self.params[i] for i in self.bucket_params[b]], b == len(self.buckets) - 1)
            self.works.append((b, self.hook(self.state, gb)))
            return
        if self.world == 1:
            return
        if self.compression == "bf16":
            c = t.to(torch.bfloat16)
            self.works.append((b, ("bf16", c, dist.all_reduce(c, async_op=True))))
        else:
            self.works.append((b, dist.all_reduce(t, async_op=True)))

    def mark_ready(self, i: int):
        if not self.open:
            self.prepare()
        if i in self.seen:
            return
        self.seen.add(i)
        b = self.bucket_of.get(i)
        if b is None:
            return
        self.pending[b] -= 1
        if self.pending[b] == 0:
            self.ready[b] = True
        while self.next < len(self.buckets) and self.ready[self.next]:
            self._launch(self.next)
            self.next += 1

    def finalize(self):
        if not self.open:
            return
        while self.next < len(self.buckets):
            self._launch(self.next)
            self.next += 1
        for b, w in self.works:
            t = self.buckets[b]
            if self.hook is not None:
                r = w.wait() if isinstance(w, torch.futures.Future) else w
                if isinstance(r, (list, tuple)):
                    r = r[0]
                if isinstance(r, torch.Tensor) and r.data_ptr() != t.data_ptr():
                    t.copy_(r)
            elif isinstance(w, tuple):  # bf16 compressed
                _, c, work = w
                work.wait()
                t.copy_(c.float().div_(self.world))
            else:
                w.wait()
                t.div_(self.world)
        self.open = False

    def last_timings(self):
        return []

    def launch_order(self):
        return list(self.order)


class _GlooTransport:
    """Collective side of the native reducer's host-transport mode (gloo control plane, CPU or
    host-staged GPU tensors): ``on_launch(b)`` issues bucket b's async all-reduce, ``on_finalize()``
    waits for all of them and averages.  The readiness tracking, index-order issue and finalize
    sequencing stay in C++ (``_C.Reducer.host``), the same code the RCCL path runs."""

    def __init__(self, buckets: List[torch.Tensor], world: int, compression: Optional[str], timing: bool = False):
        self.buckets, self.world, self.compression = buckets, world, compression
        self.works = []
        # timing: host-clock per-bucket (issue -> wait returned) times of the last step, like the RCCL
        # reducer's event timings: [(bucket, allreduce_ms, start relative to the end of backward, ms)]
        self.timing, self.timings, self._t0 = timing, [], {}
        self.t_bwd_end = None  # set by DDP._finalize (end of backward)

    def on_launch(self, b: int):
        if self.world == 1:
            return
        if self.timing:
            self._t0[b] = time.perf_counter()
        t = self.buckets[b]
        if t.is_cuda:
            _aux_wait(t.device)  # weight grads written on the side stream
        if self.compression == "bf16":
            c = t.to(torch.bfloat16)
            self.works.append((b, c, dist.all_reduce(c, async_op=True)))
        else:
            self.works.append((b, None, dist.all_reduce(t, async_op=True)))

    def on_finalize(self):
        t_end = self.t_bwd_end if self.t_bwd_end is not None else time.perf_counter()
        self.t_bwd_end = None
        timings = []
        for b, c, w in self.works:
            w.wait()
            if self.timing and b in self._t0:
                now = time.perf_counter()
                timings.append((b, 1e3 * (now - self._t0[b]), 1e3 * (self._t0[b] - t_end)))
            t = self.buckets[b]
            if c is not None:
                t.copy_(c.float().div_(self.world))
            else:
                t.div_(self.world)
        self.works = []
        if self.timing:
            self.timings, self._t0 = timings, {}


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, device_ids=None, output_device=None, broadcast_buffers: bool = True,
                 bucket_cap_mb: Optional[float] = None, first_bucket_mb: Optional[float] = None,
                 find_unused_parameters: bool = False, gradient_as_bucket_view: bool = True,
                 init_sync: bool = True, timing: bool = False, comm=None, force_comm: bool = False,
                 gradient_compression: Optional[str] = None, rebuild_buckets: bool = True,
                 debug: Optional[bool] = None, last_bucket_mb="auto", register_buckets: bool = True):
        super().__init__()
        self.module = module
        self.broadcast_buffers = broadcast_buffers
        self.find_unused_parameters = find_unused_parameters
        self.require_backward_grad_sync = True
        self.world_size = pdist.get_world_size()
        self._params = [p for p in module.parameters() if p.requires_grad]
        self._index = {id(p): i for i, p in enumerate(self._params)}
        # bucket caps: explicit values win; otherwise the 7-link xGMI policy (buckets.xgmi_bucket_policy)
        p_first, p_cap, p_last = xgmi_bucket_policy(self.world_size, 4 * sum(p.numel() for p in self._params))
        cap = int((bucket_cap_mb if bucket_cap_mb is not None else p_cap) * 1024 * 1024)
        first_mb = p_first if first_bucket_mb is None else first_bucket_mb
        first = int(first_mb * 1024 * 1024) if first_mb else cap
        self.bucket_cap_bytes, self.first_bucket_bytes = cap, first
        # the last-ready gradients (the only all-reduce that cannot overlap backward) go in
        # small buckets: at 8 GPUs only the final <= last_bucket_mb piece is exposed
        last_mb = p_last if last_bucket_mb == "auto" else last_bucket_mb
        self.last_bucket_bytes = int(last_mb * 1024 * 1024) if last_mb else None
        # DPE_REGISTER_BUCKETS=0: no ncclCommRegister of the bucket buffers (A/B, debugging)
        self._register = register_buckets and os.environ.get("DPE_REGISTER_BUCKETS", "1") != "0"
        self._comm = comm if comm is not None else pdist.comm()
        self._force = force_comm
        self._timing = timing
        if gradient_compression not in (None, "none", "bf16"):
            raise ValueError(f"gradient_compression must be None or 'bf16', got {gradient_compression!r}")
        self._compression = None if gradient_compression in (None, "none") else gradient_compression
        self._hook, self._hook_state = None, None
        self._debug = (os.environ.get("DPE_DDP_DEBUG", "0") == "1") if debug is None else debug
        # one-time rebuild from the observed ready order (c10d: after iteration 0)
        self._rebuild_pending = False
        self._rebuild_enabled = rebuild_buckets
        self._record_order = rebuild_buckets
        self._ready_order: List[int] = []
        self.bucket_rebuilds = 0
        if init_sync and self.world_size > 1:
            self._sync_module_states()
        self._flat_bufs: List[torch.Tensor] = []
        self._flat_views = []
        if broadcast_buffers and self.world_size > 1:
            self._flatten_buffers()
        self._ov_opt = None  # overlap_optimizer()
        self._budget_probe = self._budget_probe_init()
        self._build_buckets(None)
        self._queued = False
        self._hooks = []
        for i, p in enumerate(self._params):
            p._dpe_direct = True
            p._dpe_ready = self._on_ready
            self._hooks.append(p.register_post_accumulate_grad_hook(self._on_accumulated))
            if getattr(p, "_dpe_overwrite_ok", False):
                self._hooks.append(p.register_hook(self._fresh_guard(i)))

    # --------------------------------------------------------------- setup
    @torch.no_grad()
    def _sync_module_states(self):
        """Broadcast params + buffers from rank 0, one flat buffer per dtype (reference C3, C9 at init)."""
        tensors = [p.data for p in self.module.parameters()] + [b for b in self.module.buffers()]
        by_dtype = {}
        for t in tensors:
            by_dtype.setdefault((t.dtype, t.device), []).append(t)
        for (dt, dev), ts in by_dtype.items():
            flat = torch.cat([t.reshape(-1) for t in ts])
            pdist.broadcast(flat if dt != torch.bool else flat.view(torch.uint8), 0)
            off = 0
            for t in ts:
                n = t.numel()
                t.copy_(flat[off: off + n].view_as(t))
                off += n

    @torch.no_grad()
    def _build_buckets(self, order: Optional[List[int]]):
        n = len(self._params)
        if order is None:
            order = list(range(n))[::-1]
        sizes = [p.numel() * 4 for p in self._params]  # fp32 grads
        keys = [(str(p.device),) for p in self._params]
        old = None
        if getattr(self, "buckets", None) is not None:
            old = [p.grad.detach().clone() if p.grad is not None else None for p in self._params]
        self.bucket_indices = assign_buckets(sizes, order, self.bucket_cap_bytes, self.first_bucket_bytes, keys,
                                             self.last_bucket_bytes)
        self.buckets: List[torch.Tensor] = []
        self._views = {}
        for bidx in self.bucket_indices:
            total = sum(self._params[i].numel() for i in bidx)
            dev = self._params[bidx[0]].device
            buf = torch.zeros(total, dtype=torch.float32, device=dev)
            off = 0
            for i in bidx:
                p = self._params[i]
                self._views[i] = buf[off: off + p.numel()].view_as(p)
                off += p.numel()
            self.buckets.append(buf)
        for i, p in enumerate(self._params):
            p.grad = self._views[i]
            if old is not None and old[i] is not None:
                self._views[i].copy_(old[i])
        self._pbucket = [0] * n
        for b, bidx in enumerate(self.bucket_indices):
            for i in bidx:
                self._pbucket[i] = b
        self._make_reducer()
        if self._debug:
            self._check_layout()

    def _make_reducer(self):
        native_ok = self._comm is not None and self._params and self._params[0].is_cuda and self._hook is None
        if native_ok:
            from ..ops._ext import ext

            self.reducer = ext().Reducer(self.buckets, self.bucket_indices, len(self._params), self._comm, self._timing,
                                         self._force, self._compression == "bf16", self._debug, self._register)
            self._native = True
        elif self._hook is None and _has_ext():
            # gloo / CPU: the C++ reducer in host-transport mode (same sequencing as the RCCL path)
            from ..ops._ext import ext

            self._transport = _GlooTransport(self.buckets, self.world_size, self._compression, self._timing)
            self.reducer = ext().Reducer.host(self.buckets, self.bucket_indices, len(self._params), self.world_size,
                                              self._transport.on_launch, self._transport.on_finalize)
            self._native = False
        else:
            # custom comm hooks (or no native extension built): the Python reducer
            self.reducer = _PyReducer(self.buckets, self.bucket_indices, len(self._params), self._params, self._hook,
                                      self._hook_state, self._compression)
            self._native = False

    def layout_fingerprint(self) -> str:
        h = hashlib.sha1()
        for bidx, buf in zip(self.bucket_indices, self.buckets):
            h.update(repr((tuple(bidx), buf.numel(), str(buf.dtype))).encode())
        return h.hexdigest()

    def _check_layout(self):
        """Fail fast on a cross-rank bucket-layout mismatch (would otherwise hang in RCCL)."""
        if self.world_size == 1 or not dist.is_initialized():
            return
        mine = self.layout_fingerprint()
        allfp = [None] * self.world_size
        dist.all_gather_object(allfp, mine)
        if len(set(allfp)) != 1:
            raise RuntimeError(f"DDP bucket layout differs across ranks: {allfp}")

    def register_comm_hook(self, state, hook: Callable):
        """torch DDP API.  Built-in hooks run on the native reducer; custom ones on the Python reducer."""
        if hook in _hooks.BUILTIN:
            self._compression = _hooks.BUILTIN[hook]
            self._hook, self._hook_state = None, None
        else:
            self._hook, self._hook_state = hook, state
        self._make_reducer()

    def enable_timing(self, on: bool = True):
        """Per-bucket comm timing (HIP events) for the overlap / bucket-size sweep."""
        self._timing = on
        if self._native:
            self.reducer.set_timing(on)  # from the next step's prepare()
        elif getattr(self, "_transport", None) is not None:
            self._transport.timing = on

    def bucket_timings(self):
        """[(bucket, allreduce_ms, start relative to the end of backward in ms)] of the last timed step."""
        if not self._native and getattr(self, "_transport", None) is not None:
            return list(self._transport.timings)
        return self.reducer.last_timings()

    def _attach_grads(self, zero: bool):
        reattached = False
        for i, p in enumerate(self._params):
            v = self._views[i]
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                if p.grad is not None:
                    v.copy_(p.grad)
                    p.grad = v
                else:
                    p.grad = v
                    reattached = True
        if zero or reattached:
            # set_to_none=True zero_grad dropped the views: grads restart from zero (one multi-tensor
            # launch).  Parameters whose first backward writer overwrites (ops/_state.py grad_fresh)
            # are marked fresh instead of filled.
            # (GPU only: there every writer of such a parameter is one of our kernels; on the CPU
            # autograd's AccumulateGrad adds into .grad)
            ow = [getattr(p, "_dpe_overwrite_ok", False) and p.is_cuda and _GRAD_FRESH for p in self._params]
            if any(ow):
                for p, o in zip(self._params, ow):
                    p._dpe_fresh = o
                torch._foreach_zero_([self._views[i] for i, o in enumerate(ow) if not o])
            else:
                torch._foreach_zero_(list(self.buckets))

    def _fresh_guard(self, i: int):
        """Tensor hook of a ``_dpe_overwrite_ok`` parameter: it runs when autograd is about to
        accumulate a gradient for it (a writer other than our kernels, which write the bucket view
        directly and hand autograd no tensor).  If the view still holds last step's values (fresh, no
        kernel has overwritten it yet), zero it first so AccumulateGrad adds into zeros, not stale data."""
        def hook(grad):
            p = self._params[i]
            if getattr(p, "_dpe_fresh", False):
                p._dpe_fresh = False
                self._views[i].zero_()
            return grad

        return hook

    def _on_accumulated(self, p):
        """Post-accumulate-grad hook: readiness of parameters written through autograd.  It also fires
        after a node that wrote the parameter itself (and returned None for it) -- those announce
        themselves with grad_done, and a parameter whose weight gradient is still queued for a grouped
        launch (``_dpe_deferred``, models/_gpt2_fused.py) must not be announced before that launch.
        Either way every node that read the parameter has returned: for the overlapped optimizer the
        parameter may now be rewritten."""
        if self._ov_opt is not None and self.require_backward_grad_sync:
            self._ov_mark(p, 2)
        if getattr(p, "_dpe_deferred", False):
            return
        self._on_ready(p)

    # ------------------------------------------------- optimizer in backward
    def overlap_optimizer(self, optimizer, enable: bool = True) -> None:
        """Step the fused ``optimizer`` (optim.Adam / AdamW / SGD) per gradient bucket during backward,
        on a dedicated HIP stream; the training loop keeps calling ``optimizer.step()`` after backward
        (it joins the stream and steps whatever is left).  GPU only; with custom comm hooks or a host
        (gloo) transport at world > 1 the gradients are final only at the end of backward, so the
        overlap is refused there.  Gradient clipping / unscaling between backward and step cannot be
        combined with it (the update has already run)."""
        if not enable:
            if self._ov_opt is not None:
                self._ov_opt._ov_detach()
            self._ov_opt = None
            return
        if not hasattr(optimizer, "_ov_bucket_step"):
            raise TypeError("overlap_optimizer needs one of the fused optimizers (distributed_pytorch_example_amd.optim)")
        if not (self._params and self._params[0].is_cuda):
            raise RuntimeError("overlap_optimizer: GPU parameters only")
        if self.world_size > 1 and not self._native:
            raise RuntimeError("overlap_optimizer: needs the native RCCL reducer at world size > 1")
        ids = {id(p) for g in optimizer.param_groups for p in g["params"]}
        if any(id(p) not in ids for p in self._params):
            raise ValueError("overlap_optimizer: the optimizer must own every parameter DDP reduces")
        self._ov_opt = optimizer
        self._ov_stream = torch.cuda.Stream(device=self._params[0].device)
        optimizer._ov_attach(self._ov_stream)
        self._ov_reset()

    def _ov_reset(self):
        nb = len(self.bucket_indices)
        self._ov_flags = bytearray(len(self._params))  # bit 1: gradient final, bit 2: every reader returned
        self._ov_count = [0] * nb
        self._ov_next = 0

    def _ov_mark(self, p, bit: int):
        i = self._index.get(id(p))
        if i is None:
            return
        f = self._ov_flags[i]
        if f & bit:
            return
        f |= bit
        self._ov_flags[i] = f
        if f == 3:
            self._ov_count[self._pbucket[i]] += 1
            self._ov_drain(False)

    def _ov_drain(self, final: bool):
        """Step the buckets that are complete, in index order (the order the reducer issues them)."""
        launched = self.reducer.buckets_launched if hasattr(self.reducer, "buckets_launched") else len(self.buckets)
        while self._ov_next < len(self.bucket_indices):
            b = self._ov_next
            if not final and (self._ov_count[b] < len(self.bucket_indices[b]) or b >= launched):
                break
            s = self._ov_stream
            ev = torch.cuda.Event()
            ev.record()  # everything enqueued so far on the compute stream: the gradients and their readers
            s.wait_event(ev)
            dev = self._params[0].device
            aux = _state._aux_streams.get(dev.index if dev.index is not None else torch.cuda.current_device())
            if aux is not None:
                s.wait_stream(aux)
            if hasattr(self.reducer, "stream_wait_comm"):
                self.reducer.stream_wait_comm(s.cuda_stream)  # this bucket's all-reduce
            self._ov_opt._ov_bucket_step([self._params[i] for i in self.bucket_indices[b]], s)
            self._ov_next += 1

    # ---------------------------------------------------------- per-step
    def _on_ready(self, p):
        if not self.require_backward_grad_sync:
            return
        i = self._index.get(id(p))
        if i is None:
            return
        if self._record_order:
            self._ready_order.append(i)
        if not self._queued:
            self._queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
        self.reducer.mark_ready(i)
        if self._ov_opt is not None:
            self._ov_mark(p, 1)

    # ------------------------------------------------------- adaptive CU budget
    def _budget_probe_init(self):
        """The CU budget (parallel/dist.py cu_reserve_for: persistent kernels leave slots to RCCL's channel
        blocks while a bucket all-reduce is in flight) pays off only when collectives occupy a good part of
        backward.  It is in force from the first bucket launch to the end of backward, while RCCL's blocks
        are resident only during the all-reduces.  So a few steps after warm-up (steps 2 .. 1 + N,
        N = DPE_CU_BUDGET_SAMPLES, default 3) are timed with events -- forward + backward on the compute
        stream, and every bucket all-reduce on the comm stream (the reducer's own per-bucket events) -- and
        the budget is dropped when the MEASURED all-reduce time is below DPE_CU_BUDGET_MIN_DUTY (default
        0.10) of the backward (taken as 2/3 of forward + backward).  Each quantity is the minimum over the
        samples (the first timed step can still carry first-call costs), then the MAX over ranks through
        the control plane, so every rank applies the same decision (same persistent-kernel slot counts and
        split plans everywhere).  The modelled time, 2 (W-1)/W x gradient bytes / DPE_XGMI_BUS_GBPS
        (default 300), decides only if no step could be timed (``settle_cu_budget`` before any sample).
        Probe on one GPU (profiles/cu_hog_probe_r5.txt, 16 RCCL-sized workgroups resident only in the
        modelled W = 8 windows): ResNet-50 +1.9 % without the budget vs +4.8 % with it, GPT-2 +5.4 % vs
        +4.1 %.  An explicit DPE_CU_RESERVE is never changed."""
        if (self.world_size <= 1 or os.environ.get("DPE_CU_RESERVE") or os.environ.get("DPE_CU_BUDGET_ADAPT", "1") == "0"
                or not self._params or not self._params[0].is_cuda or not _has_ext()):
            return None
        from ..ops._ext import ext

        if ext().cu_reserve_config() <= 0:
            return None
        gbps = float(os.environ.get("DPE_XGMI_BUS_GBPS", "300"))
        nbytes = 4 * sum(p.numel() for p in self._params)
        comm_ms = 2.0 * (self.world_size - 1) / self.world_size * nbytes / (gbps * 1e6)
        return {"step": 0, "pending": None, "samples": [], "comm_ms_model": comm_ms,
                "nsamples": max(1, int(os.environ.get("DPE_CU_BUDGET_SAMPLES", "3"))),
                "min_duty": float(os.environ.get("DPE_CU_BUDGET_MIN_DUTY", "0.10")), "decision": None,
                "reserve": ext().cu_reserve_config()}

    def _budget_collect(self):
        """Read the timed step in flight (blocks until its collectives completed; warm-up steps only)."""
        pr = self._budget_probe
        pend, pr["pending"] = pr["pending"], None
        if pend is None:
            return
        a, b = pend
        if self._native and not self._timing:
            self.reducer.set_timing(False)
        if b is None:
            return
        b.synchronize()
        tim = self.reducer.last_timings() if self._native else []
        if tim:
            pr["samples"].append((a.elapsed_time(b), sum(t[1] for t in tim)))

    def _budget_decide(self):
        pr = self._budget_probe
        if pr["samples"]:
            fb = min(s[0] for s in pr["samples"])
            cm = min(s[1] for s in pr["samples"])
            source = "measured"
        else:
            fb, cm, source = 0.0, pr["comm_ms_model"], "model"
        v = torch.tensor([fb, cm, float(len(pr["samples"]))], dtype=torch.float64)
        if self.world_size > 1 and dist.is_initialized():
            dist.all_reduce(v, op=dist.ReduceOp.MAX)  # control plane: one decision for every rank
            m = torch.tensor([float(len(pr["samples"]))], dtype=torch.float64)
            dist.all_reduce(m, op=dist.ReduceOp.MIN)
            if m.item() == 0:  # some rank has no sample: everyone falls back to the model
                source = "model"
        fb, cm = v[0].item(), v[1].item()
        if source == "model":
            cm = pr["comm_ms_model"]
        duty = cm / max(1e-3, fb * 2.0 / 3.0) if fb > 0 else float("inf")
        keep = duty >= pr["min_duty"]
        pr["decision"] = {"source": source, "fwd_bwd_ms": round(fb, 3), "comm_ms": round(cm, 3),
                          "comm_ms_model": round(pr["comm_ms_model"], 3), "samples": len(pr["samples"]),
                          "duty": round(duty, 4) if fb > 0 else None, "min_duty": pr["min_duty"],
                          "reserve_slots": pr["reserve"], "budget": keep}
        if not keep:
            from .dist import set_cu_budget

            set_cu_budget(0)

    def _budget_probe_forward(self):
        pr = self._budget_probe
        if pr is None or pr["decision"] is not None:
            return
        pr["step"] += 1
        self._budget_collect()
        if len(pr["samples"]) >= pr["nsamples"] or pr["step"] > pr["nsamples"] + 4:
            self._budget_decide()
            return
        if pr["step"] >= 2:  # step 1: warm-up (allocator, bucket rebuild, first-call costs)
            if self._native:
                self.reducer.set_timing(True)
            a = torch.cuda.Event(enable_timing=True)
            a.record()
            pr["pending"] = [a, None]

    def _budget_probe_backward_end(self):
        pr = self._budget_probe
        if pr is not None and pr["decision"] is None and pr["pending"] is not None and pr["pending"][1] is None:
            b = torch.cuda.Event(enable_timing=True)
            b.record()
            pr["pending"][1] = b

    def settle_cu_budget(self):
        """Decide the adaptive CU budget now (collective: every rank calls it at the same point, e.g. after
        the warm-up loop) from the steps timed so far; the model decides if none was.  Returns the decision
        record (``cu_budget_info``)."""
        pr = self._budget_probe
        if pr is not None and pr["decision"] is None:
            self._budget_collect()
            self._budget_decide()
        return self.cu_budget_info()

    @property
    def cu_budget_decision(self):
        """None until decided (or when not adaptive); else the measured inputs and whether the budget stays."""
        return None if self._budget_probe is None else self._budget_probe["decision"]

    def cu_budget_info(self) -> dict:
        """The CU-budget state for reports: the adaptive decision, or why there is none."""
        if self._budget_probe is not None:
            return self._budget_probe["decision"] or {"source": "pending"}
        if self.world_size <= 1:
            return {"source": "off", "reason": "world size 1 (no collectives)", "budget": False}
        if not (self._params and self._params[0].is_cuda and _has_ext()):
            return {"source": "off", "reason": "host transport (no GPU compute kernels)", "budget": False}
        if os.environ.get("DPE_CU_RESERVE"):
            return {"source": "env", "reserve_slots": int(os.environ["DPE_CU_RESERVE"]),
                    "budget": int(os.environ["DPE_CU_RESERVE"]) > 0}
        from ..ops._ext import ext

        r = ext().cu_reserve_config()
        return {"source": "fixed", "reserve_slots": r, "budget": r > 0}

    def _finalize(self):
        self._queued = False
        self._budget_probe_backward_end()
        if getattr(self, "_transport", None) is not None and not self._native:
            self._transport.t_bwd_end = time.perf_counter()
        for i, p in enumerate(self._params):  # fresh but never written this step: zero, as stock
            if getattr(p, "_dpe_fresh", False):
                p._dpe_fresh = False
                self._views[i].zero_()
        self.reducer.finalize()
        if self._ov_opt is not None:
            self._ov_drain(True)  # backward is over: every remaining bucket (unused parameters too)
        if self._record_order:
            self._record_order = False
            self._rebuild_pending = self._rebuild_enabled

    def finish_gradient_sync(self):
        """Explicit end-of-backward hook (also queued automatically)."""
        if self.require_backward_grad_sync:
            self.reducer.finalize()
            self._queued = False

    def _rebuild_from_observed_order(self):
        seen = set()
        order = []
        for i in self._ready_order:
            if i not in seen:
                seen.add(i)
                order.append(i)
        order += [i for i in range(len(self._params))[::-1] if i not in seen]  # unused params last
        if self.world_size > 1 and dist.is_initialized():
            box = [order]
            dist.broadcast_object_list(box, src=0)  # identical buckets on every rank (C5)
            order = box[0]
        if order != list(range(len(self._params)))[::-1] or self.bucket_rebuilds == 0:
            self._build_buckets(order)
        self.bucket_rebuilds += 1
        self._rebuild_pending = False

    def forward(self, *args, **kwargs):
        if torch.is_grad_enabled():
            if self._rebuild_pending and self.require_backward_grad_sync:
                self._rebuild_from_observed_order()
            self._attach_grads(zero=False)
            for p in self._params:
                p._dpe_uses = 0
            if self.require_backward_grad_sync:
                self._budget_probe_forward()
                self.reducer.prepare()
                if self._ov_opt is not None:
                    self._ov_reset()
        if self.broadcast_buffers and self.world_size > 1:
            self._sync_buffers()
        return self.module(*args, **kwargs)

    @torch.no_grad()
    def _flatten_buffers(self):
        """Re-home every buffer -- floating (BN running stats) and integer (``num_batches_tracked``)
        alike, as stock DDP's ``broadcast_buffers`` syncs them all -- as a view of one flat tensor
        per (dtype, device): one broadcast per dtype per forward."""
        groups, seen = {}, set()
        for mod in self.module.modules():
            for name, b in mod._buffers.items():
                if b is None or id(b) in seen:
                    continue
                seen.add(id(b))
                groups.setdefault((b.dtype, b.device), []).append((mod, name, b))
        self._flat_bufs, self._flat_views = [], []
        for items in groups.values():
            flat = torch.cat([b.reshape(-1) for _, _, b in items])
            off = 0
            for mod, name, b in items:
                n = b.numel()
                v = flat[off: off + n].view_as(b)
                mod._buffers[name] = v
                self._flat_views.append((mod, name, v))
                off += n
            self._flat_bufs.append(flat)

    @torch.no_grad()
    def _sync_buffers(self):
        if not self._flat_bufs:
            return
        if any(mod._buffers.get(name) is not v for mod, name, v in self._flat_views):
            self._flatten_buffers()  # a buffer was re-assigned: re-home it
        for flat in self._flat_bufs:
            pdist.broadcast(flat if flat.dtype != torch.bool else flat.view(torch.uint8), 0)

    @contextlib.contextmanager
    def no_sync(self):
        """Accumulate gradients locally (grad-accumulation micro-steps)."""
        old = self.require_backward_grad_sync
        self.require_backward_grad_sync = False
        try:
            yield
        finally:
            self.require_backward_grad_sync = old

    # ------------------------------------------------------------- info
    def num_buckets(self) -> int:
        return len(self.buckets)

    def bucket_bytes(self) -> List[int]:
        return [b.numel() * b.element_size() for b in self.buckets]


DDP = DistributedDataParallel
