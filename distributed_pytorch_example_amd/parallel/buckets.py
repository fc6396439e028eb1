"""Gradient bucket assignment.

Semantics of c10d's ``_compute_bucket_assignment_by_size`` as DDP uses it
(`$TORCH/nn/parallel/distributed.py:1199-1206`, `$CXX/reducer.hpp:590`):
parameters are taken in the order their gradients become ready (reverse
registration order as the a-priori estimate), grouped per (dtype, device),
and a bucket is closed once it reaches its byte cap; the first bucket uses a
smaller cap (1 MiB) so the first all-reduce starts early in backward.

The MI355X default differs only in the caps the caller passes: xGMI rings are
per-link bound (7 x ~153 GB/s), so a bucket must be large enough to amortise
RCCL's launch/latency (~tens of us) yet small enough that the LAST bucket
(which cannot overlap) is short.  ``bench.py --bucket-mb`` sweeps it.
"""
from __future__ import annotations

from typing import List, Sequence


def assign_buckets(sizes_bytes: Sequence[int], order: Sequence[int], cap_bytes: int,
                   first_cap_bytes: int | None = None, keys: Sequence | None = None,
                   last_cap_bytes: int | None = None) -> List[List[int]]:
    """Return a list of buckets (lists of parameter indices, in ``order``).

    ``last_cap_bytes`` (MI355X addition, not in c10d): the final bucket -- the gradients
    that become ready last, whose all-reduce is the only one that cannot overlap
    backward -- is re-split into pieces of at most this many bytes, so all but the
    last small piece start while the earliest layers are still in backward."""
    buckets = _assign(sizes_bytes, order, cap_bytes, first_cap_bytes, keys)
    if last_cap_bytes and len(buckets) > 1:
        tail, pieces, cur, nbytes = buckets.pop(), [], [], 0
        for idx in tail:
            if cur and nbytes + sizes_bytes[idx] > last_cap_bytes:
                pieces.append(cur)
                cur, nbytes = [], 0
            cur.append(idx)
            nbytes += sizes_bytes[idx]
        if cur:
            pieces.append(cur)
        buckets.extend(pieces)
    return buckets


def _assign(sizes_bytes, order, cap_bytes, first_cap_bytes, keys) -> List[List[int]]:
    if first_cap_bytes is None:
        first_cap_bytes = cap_bytes
    buckets: List[List[int]] = []
    open_: dict = {}  # key -> (indices, bytes)
    for idx in order:
        k = keys[idx] if keys is not None else None
        cur, nbytes = open_.get(k, ([], 0))
        cur.append(idx)
        nbytes += sizes_bytes[idx]
        cap = first_cap_bytes if not buckets else cap_bytes
        if nbytes >= cap:
            buckets.append(cur)
            open_.pop(k, None)
        else:
            open_[k] = (cur, nbytes)
    for k, (cur, _) in open_.items():
        if cur:
            buckets.append(cur)
    return buckets
