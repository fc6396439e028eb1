"""DDP communication hooks (API of ``torch.distributed.algorithms.ddp_comm_hooks``).

The reference never registers one (its DDP uses the default all-reduce,
SURVEY §2.2 I4); they are provided because ``register_comm_hook`` is part of
the DDP surface a user of the reference can reach for.

* ``allreduce_hook``      -- the default: average the bucket across ranks.
* ``bf16_compress_hook``  -- all-reduce a bf16 copy of the bucket and
  decompress (half the xGMI/RoCE bytes).  On the rccl backend DDP maps both
  built-ins onto the native C++ reducer (the cast kernels and ncclAvg run on
  the communicator's stream, overlapped with backward); any other callable
  runs through the Python reducer: ``hook(state, bucket) -> Future[Tensor]``
  or a tensor, called once per bucket in bucket order, as soon as the bucket
  is complete.
"""
from __future__ import annotations

from typing import List

import torch

from . import dist as pdist


class GradBucket:
    """What a hook sees: the flat gradient buffer of one bucket and its parameters."""

    def __init__(self, index: int, buffer: torch.Tensor, params: List[torch.nn.Parameter], last: bool):
        self._index, self._buffer, self._params, self._last = index, buffer, params, last

    def index(self) -> int:
        return self._index

    def buffer(self) -> torch.Tensor:
        return self._buffer

    def is_last(self) -> bool:
        return self._last

    def parameters(self) -> List[torch.nn.Parameter]:
        return list(self._params)

    def gradients(self) -> List[torch.Tensor]:
        return [p.grad for p in self._params]


def _done(t: torch.Tensor) -> torch.futures.Future:
    fut = torch.futures.Future()
    fut.set_result(t)
    return fut


def allreduce_hook(state, bucket: GradBucket) -> torch.futures.Future:
    """Average the bucket over all ranks (in place)."""
    t = bucket.buffer()
    pdist.all_reduce(t, "avg")
    return _done(t)


def bf16_compress_hook(state, bucket: GradBucket) -> torch.futures.Future:
    """All-reduce a bf16 copy, decompress into the fp32 bucket."""
    t = bucket.buffer()
    c = t.to(torch.bfloat16)
    pdist.all_reduce(c, "avg")
    t.copy_(c)
    return _done(t)


BUILTIN = {allreduce_hook: None, bf16_compress_hook: "bf16"}
