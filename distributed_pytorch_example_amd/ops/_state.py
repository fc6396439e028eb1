"""Per-parameter runtime state shared by layers, optimizers and the DDP reducer.

* bf16 compute shadows: layers keep fp32 master parameters; the MFMA kernels
  read a bf16 copy.  The fused optimizer kernels write the shadow in the same
  pass that updates the master (no cast pass per step).  A shadow is re-cast
  whenever ``param._version`` moved (torch-side in-place edits such as
  ``load_state_dict``) -- our own kernels write through raw pointers and
  keep the version.  Shadows may be *padded* (extra trailing zero rows for
  out_features % 8 != 0); the fused optimizer then still writes the prefix.
  Shadows whose layout differs from the master (e.g. the ResNet stem's
  channel-padded filter) register a ``derive`` function that the optimizer
  re-runs after each step (``post_step`` hooks, graph-capturable).

* direct gradients: when DDP runs with gradient-as-bucket-view, our backward
  kernels accumulate weight gradients straight into ``param.grad`` (a view of
  the flat bucket) and signal readiness to the reducer themselves, instead of
  returning a fresh tensor that autograd would add into the bucket.
"""
from __future__ import annotations

import torch

_derived: list = []  # (param, shadow, fn)


def shadow(p: torch.Tensor, pad_rows: int = 0) -> torch.Tensor:
    """bf16 shadow of fp32 master ``p`` (optionally with zero pad rows)."""
    sh = getattr(p, "_dpe_shadow", None)
    rows = p.shape[0] + pad_rows
    if sh is None or sh.device != p.device or sh.shape[0] < rows:
        sh = torch.zeros((rows, *p.shape[1:]), dtype=torch.bfloat16, device=p.device)
        p._dpe_shadow = sh
        p._dpe_shadow_ver = -1
    if getattr(p, "_dpe_shadow_ver", -1) != p._version:
        from ._ext import ext

        ext().cast_bf16(p.detach().reshape(-1), sh.view(-1)[: p.numel()])
        p._dpe_shadow_ver = p._version
        bump_weight_epoch()
    # one shadow per parameter: a padded (larger) shadow also serves unpadded users
    return sh if sh.shape[0] == rows else sh[:rows]


def derived_shadow(p: torch.Tensor, key: str, fn) -> torch.Tensor:
    """A shadow derived by ``fn(p) -> bf16 tensor`` (layout change), refreshed after optimizer steps."""
    attr = "_dpe_dshadow_" + key
    sh = getattr(p, attr, None)
    stamp = (p._version, _step_counter[0])
    if sh is None or getattr(p, attr + "_stamp", None) != stamp:
        new = fn(p.detach())
        if sh is None or sh.shape != new.shape:
            sh = new
        else:
            sh.copy_(new)
        setattr(p, attr, sh)
        setattr(p, attr + "_stamp", stamp)
        if not getattr(p, attr + "_reg", False):
            _derived.append((p, attr, fn))
            setattr(p, attr + "_reg", True)
    return sh


_step_counter = [0]
_weight_epoch = [0]


def bump_weight_epoch() -> None:
    """The bf16 shadows changed: the native cached flipped filters (ops.cpp flipped()) refresh at next use."""
    _weight_epoch[0] += 1
    try:
        from ._ext import ext

        C = ext()
        if hasattr(C, "set_weight_epoch"):
            C.set_weight_epoch(_weight_epoch[0])
    except Exception:  # noqa: BLE001  (CPU-only use: no extension, nothing cached)
        pass


def after_optimizer_step(params=None) -> None:
    """Refresh derived shadows in place (called by the fused optimizers; capturable)."""
    _step_counter[0] += 1
    bump_weight_epoch()
    for p, attr, fn in _derived:
        if params is not None and p not in params:
            continue
        sh = getattr(p, attr, None)
        if sh is not None:
            sh.copy_(fn(p.detach()))
            setattr(p, attr + "_stamp", (p._version, _step_counter[0]))


# ------------------------------------------------------------ direct grads
def grad_sink(p: torch.Tensor):
    """Return (buffer, direct).  direct=True: accumulate into p.grad (bucket view)."""
    if getattr(p, "_dpe_direct", False) and p.grad is not None:
        return p.grad, True
    return torch.zeros_like(p, dtype=torch.float32), False


def grad_fresh(p: torch.Tensor) -> bool:
    """True (once) when ``p.grad`` holds stale values this step's first writer must overwrite.

    DDP re-zeroes the gradient buckets at the first forward after ``zero_grad(set_to_none=True)``;
    parameters marked ``_dpe_overwrite_ok`` (every backward writes them through a kernel that honours
    this flag, the first writer overwriting) are left out of that fill -- for GPT-2-small that is
    497 MB of fp32 zeros per step plus the read of them by the weight-grad GEMMs' accumulate
    epilogues.  The flag is cleared by the first query, so later writers (a tied weight's second
    use, gradient-accumulation micro-steps) accumulate.  DDP zeroes any parameter still fresh at the
    end of backward (an unused one) before its bucket is reduced."""
    if getattr(p, "_dpe_fresh", False):
        p._dpe_fresh = False
        return True
    return False


def grad_done(p: torch.Tensor, direct: bool) -> None:
    if not direct:
        return
    uses = getattr(p, "_dpe_uses", 1)
    uses -= 1
    p._dpe_uses = uses
    if uses <= 0:
        cb = getattr(p, "_dpe_ready", None)
        if cb is not None:
            cb(p)


def note_use(p: torch.Tensor) -> None:
    """Forward-side use counter so a weight used k times is 'ready' after k backward writes.

    Called from autograd Functions' forward, which always runs with grad mode off -- so the counter
    must not depend on torch.is_grad_enabled() (it did: every counter stayed 0 and a tied weight such
    as GPT-2's wte was announced ready after its FIRST backward write, letting its bucket's all-reduce
    start before the second write; caught by the world-2 RCCL GPT-2 test).  DDP.forward resets the
    counters before every training forward, so counts left by no-grad (eval) forwards are harmless."""
    if getattr(p, "_dpe_direct", False):
        p._dpe_uses = getattr(p, "_dpe_uses", 0) + 1


# --------------------------------------------------- weight-grad side stream
# Weight gradients depend on nothing downstream in backward: they run on a side
# HIP stream so the MFMA-bound wgrad GEMMs overlap the memory-bound BatchNorm
# backward passes and the data-grad chain on the main stream.  Every gradient
# is written either on the main stream or on this one; the reducers make the
# RCCL stream wait on both before a bucket is reduced, and the end of backward
# joins the side stream back into the main one (autograd engine callback).
# Off: measured 2 % SLOWER on ResNet-50 / MI355X at batch 512 (46.6 vs 47.6 ms/step): the
# concurrent kernels contend more than they overlap.  set_wgrad_stream(True) keeps the path
# testable (tests/test_comm_gpu.py: the reducer waits on this stream too).
_WGRAD_STREAM_ON = __import__("os").environ.get("DPE_WGRAD_STREAM", "0") == "1"  # (A/B)


def set_wgrad_stream(on: bool) -> bool:
    """Enable / disable the weight-grad side stream at run time; returns the previous setting."""
    global _WGRAD_STREAM_ON
    prev, _WGRAD_STREAM_ON = _WGRAD_STREAM_ON, bool(on)
    return prev
_aux_streams: dict = {}
_aux_join_gen = [None]  # autograd graph task that already has a join queued


# K-split weight-grad slab reductions (hgemm_finalize: memory-bound, ~13 us each, 48 per GPT-2 step)
# on the side stream, co-resident with the next compute-bound GEMM on the main stream
# (DPE_FINALIZE_STREAM=1 / set_finalize_stream; A/B in docs/perf_notes.md).
_FIN_STREAM_ON = __import__("os").environ.get("DPE_FINALIZE_STREAM", "0") == "1"


def set_finalize_stream(on: bool) -> bool:
    global _FIN_STREAM_ON
    prev, _FIN_STREAM_ON = _FIN_STREAM_ON, bool(on)
    return prev


def aux_stream(device: torch.device, force: bool = False):
    """The weight-grad side stream of ``device`` (None when disabled)."""
    if not (_WGRAD_STREAM_ON or force) or device.type != "cuda":
        return None
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _aux_streams.get(idx)
    if s is None:
        s = torch.cuda.Stream(device=idx)
        _aux_streams[idx] = s
        from ._ext import ext

        ext().set_aux_stream(idx, s.cuda_stream)
    return s


def _join_aux():
    for idx, s in _aux_streams.items():
        torch.cuda.current_stream(idx).wait_stream(s)


def run_on_aux(device: torch.device, fn, *tensors):
    """Enqueue ``fn()`` on the side stream after everything already queued on the
    current stream; ``tensors`` (read by fn, allocated on the main stream) are
    kept alive for it.  Falls back to the current stream when disabled."""
    s = aux_stream(device)
    if s is None:
        return fn()
    main = torch.cuda.current_stream(device)
    s.wait_stream(main)
    with torch.cuda.stream(s):
        out = fn()
    for t in tensors:
        if t is not None:
            t.record_stream(s)
    _queue_join()
    return out


def _queue_join():
    # one join per backward pass: keyed on the running graph task (a raised backward
    # cannot leave a stale "already queued" flag behind)
    gen = torch._C._current_graph_task_id() if hasattr(torch._C, "_current_graph_task_id") else None
    if gen is None or gen != _aux_join_gen[0]:
        _aux_join_gen[0] = gen
        torch.autograd.Variable._execution_engine.queue_callback(_join_aux)


def finalize_stream(device: torch.device) -> int:
    """HIP stream handle for the slab reductions of K-split weight grads whose gradient lands in a
    DDP bucket view (0: run them on the current stream).  The reducer waits for this stream before
    a bucket's all-reduce and the end of backward joins it (so the optimizer sees the sums)."""
    if not _FIN_STREAM_ON or device.type != "cuda":
        return 0
    s = aux_stream(device, force=True)
    _queue_join()
    return s.cuda_stream


def aux_wait(device: torch.device) -> None:
    """Make the current stream wait for the side stream's queued work (Python reducer)."""
    s = _aux_streams.get(device.index if device.index is not None else torch.cuda.current_device())
    if s is not None:
        torch.cuda.current_stream(device).wait_stream(s)
