"""Distributed sampler, bit-exact with ``torch.utils.data.DistributedSampler``.

Reference use: `train.py:104-106` (shuffle=True, seed=0, drop_last=False) and
`train.py:267` (``set_epoch``).  Semantics reproduced from
`$TORCH/utils/data/distributed.py:98-134`:

* ``num_samples = ceil(N / W)`` (or ``floor`` with drop_last),
  ``total_size = num_samples * W``;
* permutation = ``torch.randperm(N, generator=manual_seed(seed + epoch))``
  on a CPU generator (so index streams match the reference exactly);
* padding wraps the head of the permutation; rank r takes ``[r::W]``.

Unlike the torch version the index list is also available as an int64 tensor
(``indices_tensor``) so the device-resident loader can gather a whole epoch's
batches on the GPU without Python-side per-sample work.
"""
from __future__ import annotations

import math
from typing import Iterator, Optional

import torch


class DistributedSampler(torch.utils.data.Sampler):
    def __init__(
        self,
        dataset,
        num_replicas: Optional[int] = None,
        rank: Optional[int] = None,
        shuffle: bool = True,
        seed: int = 0,
        drop_last: bool = False,
    ) -> None:
        if num_replicas is None or rank is None:
            import torch.distributed as dist

            if not dist.is_available() or not dist.is_initialized():
                raise RuntimeError("num_replicas/rank required when no process group is initialized")
            num_replicas = dist.get_world_size() if num_replicas is None else num_replicas
            rank = dist.get_rank() if rank is None else rank
        if rank >= num_replicas or rank < 0:
            raise ValueError(f"Invalid rank {rank}, rank should be in the interval [0, {num_replicas - 1}]")
        self.dataset = dataset
        self.num_replicas = int(num_replicas)
        self.rank = int(rank)
        self.epoch = 0
        self.drop_last = drop_last
        self.shuffle = shuffle
        self.seed = seed
        n = len(dataset)
        if drop_last and n % self.num_replicas != 0:
            self.num_samples = math.ceil((n - self.num_replicas) / self.num_replicas)
        else:
            self.num_samples = math.ceil(n / self.num_replicas)
        self.total_size = self.num_samples * self.num_replicas

    def indices_tensor(self) -> torch.Tensor:
        n = len(self.dataset)
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(n, generator=g)
        else:
            idx = torch.arange(n)
        if not self.drop_last:
            pad = self.total_size - n
            if pad > 0:
                reps = math.ceil(pad / n)
                idx = torch.cat([idx] + [idx] * reps)[: self.total_size] if pad > n else torch.cat([idx, idx[:pad]])
        else:
            idx = idx[: self.total_size]
        assert idx.numel() == self.total_size
        out = idx[self.rank : self.total_size : self.num_replicas]
        assert out.numel() == self.num_samples
        return out

    def __iter__(self) -> Iterator[int]:
        return iter(self.indices_tensor().tolist())

    def __len__(self) -> int:
        return self.num_samples

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch
