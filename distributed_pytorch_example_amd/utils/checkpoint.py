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
broadcast to every rank over the control-plane process group; all ranks
therefore resume identical state at the same epoch.  ``async_save`` writes
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


def load_checkpoint(model, optimizer, path: str, device: torch.device, broadcast: bool = True) -> int:
    """Rank 0 reads ``path`` (weights_only), every rank receives the same state.  Returns the epoch."""
    distributed = broadcast and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    rank = dist.get_rank() if distributed else 0
    ckpt: Optional[dict] = None
    if rank == 0:
        ckpt = torch.load(path, map_location="cpu", weights_only=True)
    if distributed:
        box = [ckpt]
        dist.broadcast_object_list(box, src=0)
        ckpt = box[0]
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
