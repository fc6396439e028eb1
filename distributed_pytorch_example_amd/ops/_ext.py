"""Loader for the native extension (``_C.so``, built in-tree by ``_build.py``).

Policy: GPU tensors ALWAYS go through the HIP kernels.  If the extension is
missing or fails to load, GPU ops raise -- there is no silent eager-PyTorch
fallback on the device path.  CPU tensors use the torch reference math (the
reference's CPU/gloo configuration and the CPU test suite).
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys

_C = None
_err: Exception | None = None


def _load():
    global _C, _err
    if _C is not None or _err is not None:
        return
    try:
        import torch  # noqa: F401  (loads torch's HIP/RCCL runtimes first)

        alt = os.environ.get("DPE_EXT_SO")
        if alt:  # A/B of a compile-time variant (``_build.build_variant``), same module name
            spec = importlib.util.spec_from_file_location("distributed_pytorch_example_amd._C", alt)
            _C = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(_C)
            sys.modules["distributed_pytorch_example_amd._C"] = _C
        else:
            _C = importlib.import_module("distributed_pytorch_example_amd._C")
    except Exception as e:  # pragma: no cover - exercised only when not built
        if os.environ.get("DPE_AUTOBUILD", "0") == "1":
            from .. import _build

            _build.build(verbose=False)
            _C = importlib.import_module("distributed_pytorch_example_amd._C")
        else:
            _err = e


def has_ext() -> bool:
    _load()
    return _C is not None


def ext():
    _load()
    if _C is None:
        raise RuntimeError(
            "distributed_pytorch_example_amd native extension is not built/loadable "
            f"({_err!r}). Build it with `python -m distributed_pytorch_example_amd._build`."
        )
    return _C


def on_gpu(t) -> bool:
    return t.is_cuda
