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

from typing import List, Sequence, Tuple

MiB = 1024 * 1024


def xgmi_bucket_policy(world_size: int, grad_bytes: int, alpha_s: float = 15e-6,
                       bus_bytes_per_s: float = 6.0e11) -> Tuple[float, float, float]:
    """Default (first_mb, cap_mb, last_mb) for DDP on one MI355X node (7 xGMI links per GPU).

    * cap: an all-reduce of S bytes over W ranks costs ~ alpha + 2(W-1)/W * S / B.  With RCCL's
      per-collective latency alpha ~ 15 us and a bus rate B ~ 600 GB/s per GPU (all 7 links busy
      through RCCL's multi-channel rings; SURVEY §5.8's 7 x 153 GB/s raw), the bandwidth term
      dominates (>= 4 alpha, >= 80 % link efficiency) from S ~ 21 MB at W = 8.  Fewer, larger
      buckets also mean fewer ring start-ups competing with backward kernels for CUs.  But at
      least 4 buckets keep the first all-reduces early in backward, so
      cap = clamp(grad_bytes / 4, 16 MiB, 64 MiB): ResNet-50's 102 MB of fp32 grads -> 24 MiB
      buckets, GPT-2-small's 498 MB -> 64 MiB.
    * first: 1 MiB (c10d's default): the first-ready gradients (classifier / LM head side)
      start the comm stream as early as possible.
    * last: the final bucket is the only all-reduce that cannot overlap backward; re-split into
      <= 2 MiB pieces its exposed part is ~ alpha + 2*7/8*2 MiB / B ~ 21 us at W = 8.
    At world size 1 nothing is communicated; the same layout is returned for uniformity.
    These are model numbers for a node this repository has not measured at 8 ranks; the
    bucket sweep (``scripts/sweep_buckets.sh``, ``bench.py --bucket-mb``) is the check."""
    w = max(int(world_size), 2)
    min_cap = 4 * alpha_s * bus_bytes_per_s * w / (2.0 * (w - 1))  # >= 80 % bandwidth-bound
    cap = min(max(grad_bytes / 4.0, max(16 * MiB, min_cap)), 64 * MiB)
    return 1.0, cap / MiB, 2.0


def assign_buckets(sizes_bytes: Sequence[int], order: Sequence[int], cap_bytes: int,
                   first_cap_bytes: int | None = None, keys: Sequence | None = None,
                   last_cap_bytes: int | None = None, last_pieces: int = 2) -> List[List[int]]:
    """Return a list of buckets (lists of parameter indices, in ``order``).

    ``last_cap_bytes`` (MI355X addition, not in c10d): the gradients that become ready
    LAST -- whose all-reduce is the only one that cannot overlap backward -- are peeled
    off the final bucket into ``last_pieces`` pieces of at most this many bytes, so only
    the last small piece is exposed after backward."""
    buckets = _assign(sizes_bytes, order, cap_bytes, first_cap_bytes, keys)
    if last_cap_bytes and len(buckets) > 1:
        # peel the LAST-ready gradients of the tail bucket off into `last_pieces` pieces of
        # <= last_cap_bytes; the rest of the tail stays one bucket (each extra collective costs
        # RCCL's per-call latency, so only the part that is exposed after backward is split)
        tail, pieces, cur, nbytes = buckets.pop(), [], [], 0
        rest = list(tail)
        while rest and len(pieces) < last_pieces:
            idx = rest[-1]
            if cur and nbytes + sizes_bytes[idx] > last_cap_bytes:
                pieces.append(cur)
                cur, nbytes = [], 0
                continue
            cur.insert(0, rest.pop())
            nbytes += sizes_bytes[idx]
        if cur and len(pieces) < last_pieces:
            pieces.append(cur)
        elif cur:
            rest.extend(cur)
        if rest:
            buckets.append(rest)
        buckets.extend(reversed(pieces))
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
