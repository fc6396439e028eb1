"""Fault injection for failure-detection tests.

``DPE_FAULT_INJECT="<rank>:<epoch>:<batch>[:kill|:raise]"`` makes that rank
die at that point of training: ``kill`` = SIGKILL itself (an abrupt worker
loss, as `kill -9` in the survey's experiment), ``raise`` = a Python
exception (recorded in the launcher's error file).  The launcher must then
tear the job down (fail-fast) instead of hanging in a collective.
"""
from __future__ import annotations

import os
import signal


def _spec():
    s = os.environ.get("DPE_FAULT_INJECT")
    if not s:
        return None
    parts = s.split(":")
    rank, epoch, batch = int(parts[0]), int(parts[1]), int(parts[2])
    mode = parts[3] if len(parts) > 3 else "kill"
    return rank, epoch, batch, mode


def maybe_inject(epoch: int, batch: int) -> None:
    sp = _spec()
    if sp is None:
        return
    rank, e, b, mode = sp
    if int(os.environ.get("RANK", "0")) != rank or epoch != e or batch != b:
        return
    if mode == "raise":
        raise RuntimeError(f"injected fault at rank {rank} epoch {e} batch {b}")
    os.kill(os.getpid(), signal.SIGKILL)
