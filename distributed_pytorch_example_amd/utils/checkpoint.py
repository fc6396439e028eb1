"""Checkpoint save / load, schema-compatible with the reference.

Reference: `save_checkpoint` (`train.py:178-193`) writes
``{"epoch", "model_state_dict", "optimizer_state_dict", "loss"}`` with
``torch.save``; `load_checkpoint` (`train.py:196-209`) restores model and
optimizer and returns the saved epoch (which the caller re-runs).

Compatibility: files written here load with stock
``torch.load(weights_only=True)`` (tensors / dicts / lists / numbers only)
and the optimizer state matches torch's Adam/SGD layout, so checkpoints
interchange with the reference in both directions.

Fixes for the two hazards the survey found:
  1. the resume file was opened per rank (only rank 0 ever writes it), and
  2. it was loaded *after* DDP's initial broadcast, so ranks could diverge.
Here rank 0 alone reads the file and the model/optimizer state and epoch are
broadcast to every rank (tensor bytes as one flat buffer per dtype over RCCL,
only the small skeleton through the control plane); all ranks therefore
resume identical state at the same epoch.  ``async_save`` writes
from a background thread after snapshotting tensors to host memory.
"""
from __future__ import annotations

import os
import threading
from typing import Optional

import torch
import torch.distributed as dist

from .logging import get_logger

log = get_logger("__main__")

_pending: list = []


def _standalone(obj, to_cpu: bool = False):
    """Detach + clone tensors that are views of larger storages (e.g. flat optimizer
    step counters) so the file holds plain tensors; optionally move to host."""
    if torch.is_tensor(obj):
        t = obj.detach()
        if to_cpu:
            t = t.to("cpu", copy=True)
        elif t.untyped_storage().nbytes() != t.numel() * t.element_size() or not t.is_contiguous():
            t = t.clone()
        return t
    if isinstance(obj, dict):
        return type(obj)((k, _standalone(v, to_cpu)) for k, v in obj.items())
    if isinstance(obj, list):
        return [_standalone(v, to_cpu) for v in obj]
    if isinstance(obj, tuple):
        return tuple(_standalone(v, to_cpu) for v in obj)
    return obj


def unwrap(model):
    return model.module if hasattr(model, "module") else model


def make_checkpoint(model, optimizer, epoch: int, loss: float, to_cpu: bool = False) -> dict:
    return {
        "epoch": epoch,
        "model_state_dict": _standalone(unwrap(model).state_dict(), to_cpu),
        "optimizer_state_dict": _standalone(optimizer.state_dict(), to_cpu),
        "loss": loss,
    }


def save_checkpoint(model, optimizer, epoch: int, loss: float, path: str, async_save: bool = False) -> None:
    ckpt = make_checkpoint(model, optimizer, epoch, loss, to_cpu=async_save)
    if async_save:
        wait_pending()
        th = threading.Thread(target=_write, args=(ckpt, path), daemon=True)
        th.start()
        _pending.append(th)
    else:
        _write(ckpt, path)


def _write(ckpt, path):
    tmp = path + ".tmp"
    torch.save(ckpt, tmp)
    os.replace(tmp, path)  # atomic: a crash never leaves a torn checkpoint
    log.info(f"Checkpoint saved to {path}")


def wait_pending() -> None:
    while _pending:
        _pending.pop().join()


class _TRef:
    """Placeholder for tensor #i of a broadcast checkpoint (shape / dtype / 0-d host scalar)."""

    __slots__ = ("i", "shape", "dtype", "host")

    def __init__(self, i, shape, dtype, host):
        self.i, self.shape, self.dtype, self.host = i, shape, dtype, host

    def __reduce__(self):
        return (_TRef, (self.i, self.shape, self.dtype, self.host))


def _split_tensors(obj, out: list):
    if torch.is_tensor(obj):
        out.append(obj)
        return _TRef(len(out) - 1, tuple(obj.shape), str(obj.dtype).replace("torch.", ""), obj.dim() == 0)
    if isinstance(obj, dict):
        return type(obj)((k, _split_tensors(v, out)) for k, v in obj.items())
    if isinstance(obj, list):
        return [_split_tensors(v, out) for v in obj]
    if isinstance(obj, tuple):
        return tuple(_split_tensors(v, out) for v in obj)
    return obj


def _join_tensors(obj, tensors: list):
    if isinstance(obj, _TRef):
        return tensors[obj.i]
    if isinstance(obj, dict):
        return type(obj)((k, _join_tensors(v, tensors)) for k, v in obj.items())
    if isinstance(obj, list):
        return [_join_tensors(v, tensors) for v in obj]
    if isinstance(obj, tuple):
        return tuple(_join_tensors(v, tensors) for v in obj)
    return obj


# dtypes RCCL reduces / broadcasts natively (comm.cpp to_nccl); anything else (bool, complex, fp8,
# uint16, ...) crosses the wire as a byte view of the same flat buffer and keeps its dtype
_WIRE_DTYPES = (torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int32, torch.int64, torch.uint8,
                torch.int8)


def broadcast_state(ckpt: Optional[dict], device: torch.device) -> dict:
    """Rank 0's checkpoint to every rank: the tensor-free skeleton (keys, shapes, dtypes, numbers)
    through the control plane, the tensor bytes as ONE flat buffer per dtype through
    ``parallel.dist.broadcast`` -- RCCL over xGMI on GPU jobs, not a pickle through gloo."""
    from ..parallel import dist as pdist

    rank = dist.get_rank()
    tensors: list = []
    skel = _split_tensors(ckpt, tensors) if rank == 0 else None
    box = [skel]
    dist.broadcast_object_list(box, src=0)
    skel = box[0]
    refs: list = []
    _collect_refs(skel, refs)
    refs.sort(key=lambda r: r.i)
    out = [None] * len(refs)
    by_dtype: dict = {}
    for r in refs:
        by_dtype.setdefault(r.dtype, []).append(r)
    for dt, rs in by_dtype.items():
        tdt = getattr(torch, dt)
        numels = [int(torch.Size(r.shape).numel()) for r in rs]
        total = sum(numels)
        if rank == 0:
            flat = torch.cat([tensors[r.i].reshape(-1) for r in rs]).to(device) if total else \
                torch.empty(0, dtype=tdt, device=device)
        else:
            flat = torch.empty(total, dtype=tdt, device=device)
        if total:
            pdist.broadcast(flat if tdt in _WIRE_DTYPES else flat.view(torch.uint8), 0)  # e.g. bool: as bytes
        off = 0
        for r, n in zip(rs, numels):
            t = flat[off: off + n].view(r.shape).clone()
            out[r.i] = t.cpu() if r.host else t  # 0-d (optimizer step counters) stay host scalars
            off += n
    return _join_tensors(skel, out)


def _collect_refs(obj, refs: list):
    if isinstance(obj, _TRef):
        refs.append(obj)
    elif isinstance(obj, dict):
        for v in obj.values():
            _collect_refs(v, refs)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            _collect_refs(v, refs)


def load_checkpoint(model, optimizer, path: str, device: torch.device, broadcast: bool = True) -> int:
    """Rank 0 reads ``path`` (weights_only), every rank receives the same state.  Returns the epoch."""
    distributed = broadcast and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    rank = dist.get_rank() if distributed else 0
    ckpt: Optional[dict] = None
    if rank == 0:
        ckpt = torch.load(path, map_location="cpu", weights_only=True)
    if distributed:
        ckpt = broadcast_state(ckpt, device)
    unwrap(model).load_state_dict(ckpt["model_state_dict"])
    if optimizer is not None:
        optimizer.load_state_dict(ckpt["optimizer_state_dict"])
    log.info(f"Checkpoint loaded from {path}, epoch {ckpt['epoch']}")
    return ckpt["epoch"]


def resume_exists(path: Optional[str]) -> bool:
    """Rank 0 decides whether the resume file exists and tells everyone (fix for hazard 1)."""
    if not path:
        return False
    exists = os.path.exists(path)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        t = torch.tensor([1 if exists else 0], dtype=torch.int64)
        dist.broadcast(t, 0)
        exists = bool(t.item())
    return exists
