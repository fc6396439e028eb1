"""Data-loader factory (reference `create_data_loader`, `train.py:101-116`).

Returns ``(loader, sampler)`` like the reference.  ``mode="torch"`` builds the
reference's DataLoader(num_workers=2, pin_memory=cuda) path for API parity;
``mode="device"`` (default on GPU) builds the HBM-resident `DeviceLoader`.
"""
from __future__ import annotations

import torch
from torch.utils.data import DataLoader

from .sampler import DistributedSampler
from .synthetic import DeviceLoader


def create_data_loader(dataset, batch_size: int, rank: int, world_size: int, *, shuffle: bool = True,
                       seed: int = 0, mode: str = "auto", device=None, num_workers: int = 2):
    sampler = DistributedSampler(dataset, num_replicas=world_size, rank=rank, shuffle=shuffle, seed=seed)
    if mode == "auto":
        mode = "device" if (device is not None and torch.device(device).type == "cuda") else "torch"
    if mode == "device":
        loader = DeviceLoader(dataset, batch_size, sampler=sampler, device=device)
    elif mode == "torch":
        loader = DataLoader(dataset, batch_size=batch_size, sampler=sampler, num_workers=num_workers,
                            pin_memory=torch.cuda.is_available())
    else:
        raise ValueError(f"unknown loader mode {mode!r}")
    return loader, sampler
