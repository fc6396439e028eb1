"""Synthetic datasets and the device-resident loader.

`SyntheticDataset` keeps the reference's semantics (`train.py:53-67`): the
whole dataset is materialised eagerly as ``randn(N, *shape)`` plus
``randint(0, C, (N,))`` labels.  The reference leaves it unseeded (every rank
and run differs); we keep that as the default and add an optional ``seed``.

`DeviceLoader` replaces the reference's DataLoader(num_workers=2,
pin_memory) + per-batch ``.to(device)`` (`train.py:108-114,133`): the dataset
lives in HBM (288 GB per MI355X leaves ample room), each epoch's sampler
indices are uploaded once, and each batch is a single on-device gather
(`index_select`) — no worker processes, no pinned staging, no per-batch H2D.
The batch order and contents are identical to the DataLoader path
(same sampler, same batch boundaries, last partial batch kept).
"""
from __future__ import annotations

from typing import Iterator, Optional, Sequence, Tuple

import torch
from torch.utils.data import Dataset


class SyntheticDataset(Dataset):
    def __init__(
        self,
        num_samples: int = 10000,
        input_size: int | Sequence[int] = 784,
        num_classes: int = 10,
        seed: Optional[int] = None,
        dtype: torch.dtype = torch.float32,
        device: torch.device | str = "cpu",
    ) -> None:
        self.num_samples = num_samples
        self.input_shape = (input_size,) if isinstance(input_size, int) else tuple(input_size)
        self.input_size = input_size
        self.num_classes = num_classes
        g = None
        if seed is not None:
            g = torch.Generator(device="cpu")
            g.manual_seed(seed)
        # Generate on CPU (reference RNG stream), then move once.
        data = torch.randn((num_samples, *self.input_shape), generator=g)
        labels = torch.randint(0, num_classes, (num_samples,), generator=g)
        self.data = data.to(device=device, dtype=dtype)
        self.labels = labels.to(device=device)

    def __len__(self) -> int:
        return self.num_samples

    def __getitem__(self, idx):
        return self.data[idx], self.labels[idx]


class SyntheticTokens(Dataset):
    """Token sequences for GPT-style models: ``(x[t], y[t]) = (tok[t], tok[t+1])``."""

    def __init__(self, num_samples: int, seq_len: int, vocab_size: int, seed: Optional[int] = None,
                 device: torch.device | str = "cpu") -> None:
        g = None
        if seed is not None:
            g = torch.Generator(device="cpu")
            g.manual_seed(seed)
        toks = torch.randint(0, vocab_size, (num_samples, seq_len + 1), generator=g)
        self.tokens = toks.to(device)
        self.num_samples = num_samples
        self.seq_len = seq_len

    def __len__(self) -> int:
        return self.num_samples

    def __getitem__(self, idx):
        t = self.tokens[idx]
        return t[..., :-1], t[..., 1:]


class DeviceLoader:
    """Batches a device-resident dataset by sampler order with one gather per batch."""

    def __init__(self, dataset, batch_size: int, sampler=None, drop_last: bool = False,
                 device: torch.device | str | None = None, dtype: torch.dtype | None = None) -> None:
        self.dataset = dataset
        self.batch_size = batch_size
        self.sampler = sampler
        self.drop_last = drop_last
        if isinstance(dataset, SyntheticTokens):
            self._x = dataset.tokens
            self._y = None
        else:
            self._x = dataset.data
            self._y = dataset.labels
        dev = torch.device(device) if device is not None else self._x.device
        if self._x.device != dev or (dtype is not None and self._x.dtype != dtype and self._x.is_floating_point()):
            self._x = self._x.to(device=dev, dtype=dtype if (dtype is not None and self._x.is_floating_point()) else None)
            if self._y is not None:
                self._y = self._y.to(dev)
        self.device = dev

    def __len__(self) -> int:
        n = len(self.sampler) if self.sampler is not None else len(self.dataset)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def _epoch_indices(self) -> torch.Tensor:
        if self.sampler is not None and hasattr(self.sampler, "indices_tensor"):
            idx = self.sampler.indices_tensor()
        elif self.sampler is not None:
            idx = torch.tensor(list(iter(self.sampler)), dtype=torch.long)
        else:
            idx = torch.arange(len(self.dataset))
        return idx.to(self.device, non_blocking=True)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        idx = self._epoch_indices()
        n = idx.numel()
        nb = len(self)
        for b in range(nb):
            sl = idx[b * self.batch_size: min(n, (b + 1) * self.batch_size)]
            if self._y is None:
                t = self._x.index_select(0, sl)
                yield t[:, :-1], t[:, 1:]
            else:
                yield self._x.index_select(0, sl), self._y.index_select(0, sl)
