"""DistributedSampler bit-exactness and the batch-count oracles of SURVEY §4.3."""
import pytest
import torch
from torch.utils.data.distributed import DistributedSampler as TorchSampler

from distributed_pytorch_example_amd.data import DeviceLoader, DistributedSampler, SyntheticDataset, create_data_loader


@pytest.mark.parametrize("n", [10, 97, 1000, 10000])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8, 16])
@pytest.mark.parametrize("shuffle", [True, False])
def test_bit_exact_with_torch(n, world, shuffle):
    ds = list(range(n))
    for rank in range(world):
        for epoch in (0, 1, 5):
            a = DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=shuffle, seed=0)
            b = TorchSampler(ds, num_replicas=world, rank=rank, shuffle=shuffle, seed=0)
            a.set_epoch(epoch)
            b.set_epoch(epoch)
            assert list(a) == list(b)
            assert len(a) == len(b)


def test_index_oracle():
    s = DistributedSampler(range(10), num_replicas=2, rank=0, shuffle=True, seed=0)
    assert list(s) == [4, 7, 3, 0, 6]
    s.set_epoch(1)
    assert list(s) == [5, 1, 0, 9, 7]


@pytest.mark.parametrize("world,train_b,train_pad,val_b,val_pad", [
    (1, 157, 0, 16, 0), (2, 79, 0, 8, 0), (3, 53, 2, 6, 2), (4, 40, 0, 4, 0), (8, 20, 0, 2, 0), (16, 10, 0, 1, 8)])
def test_batch_count_oracle(world, train_b, train_pad, val_b, val_pad):
    tr, va = list(range(10000)), list(range(1000))
    s = DistributedSampler(tr, num_replicas=world, rank=0)
    assert -(-len(s) // 64) == train_b and s.total_size - 10000 == train_pad
    v = DistributedSampler(va, num_replicas=world, rank=0)
    assert -(-len(v) // 64) == val_b and v.total_size - 1000 == val_pad


def test_drop_last():
    a = DistributedSampler(range(11), num_replicas=3, rank=2, drop_last=True)
    b = TorchSampler(range(11), num_replicas=3, rank=2, drop_last=True)
    assert list(a) == list(b)


def test_synthetic_dataset_semantics():
    ds = SyntheticDataset(100, 784, 10)
    x, y = ds[3]
    assert x.shape == (784,) and y.dtype == torch.int64 and 0 <= int(y) < 10
    a, b = SyntheticDataset(50, 8, 10, seed=1), SyntheticDataset(50, 8, 10, seed=1)
    assert torch.equal(a.data, b.data) and torch.equal(a.labels, b.labels)


def test_device_loader_matches_dataloader_order():
    ds = SyntheticDataset(203, 16, 10, seed=3)
    dl, s1 = create_data_loader(ds, 64, rank=1, world_size=2, mode="torch", num_workers=0)
    dv, s2 = create_data_loader(ds, 64, rank=1, world_size=2, mode="device", device="cpu")
    for e in (0, 1):
        s1.set_epoch(e)
        s2.set_epoch(e)
        got = list(dv)
        ref = list(dl)
        assert len(got) == len(ref) == len(dv)
        for (xa, ya), (xb, yb) in zip(got, ref):
            assert torch.equal(xa, xb) and torch.equal(ya, yb)
