"""roctx ranges for rocprofv3 (``--marker-trace``) around the training phases.

SURVEY §5.1: forward / backward / optimizer / per-bucket communication ranges
so a timeline shows how RCCL overlaps backward.  Uses ``libroctx64`` through
ctypes (no-op when absent or disabled); enable with ``DPE_ROCTX=1`` or
``enable(True)``.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

_lib = None
_enabled = os.environ.get("DPE_ROCTX", "0") == "1"


def _load():
    global _lib
    if _lib is None:
        for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                _lib = ctypes.CDLL(name)
                _lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                _lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                break
            except OSError:
                continue
        if _lib is None:
            _lib = False
    return _lib


def enable(on: bool = True) -> bool:
    """Turn ranges on; returns whether libroctx64 is available."""
    global _enabled
    _enabled = on
    return bool(_load()) if on else False


def push(name: str) -> None:
    if _enabled and _load():
        _lib.roctxRangePushA(name.encode())


def pop() -> None:
    if _enabled and _load():
        _lib.roctxRangePop()


def mark(name: str) -> None:
    if _enabled and _load():
        _lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def range(name: str):  # noqa: A001  (mirrors torch.cuda.nvtx.range)
    push(name)
    try:
        yield
    finally:
        pop()
