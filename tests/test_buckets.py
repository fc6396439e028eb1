"""Gradient bucket assignment (SURVEY §2.2 I5 oracles)."""
from distributed_pytorch_example_amd.models import SimpleNet, resnet50
from distributed_pytorch_example_amd.parallel import assign_buckets


def _sizes(model):
    return [p.numel() * 4 for p in model.parameters()]


def test_simplenet_is_one_bucket_of_1077288_bytes():
    s = _sizes(SimpleNet())
    order = list(range(len(s)))[::-1]
    b = assign_buckets(s, order, 25 * 2**20, 2**20)
    assert len(b) == 1 and sum(s[i] for i in b[0]) == 1077288
    assert b[0] == [5, 4, 3, 2, 1, 0]


def test_caps_and_coverage():
    s = _sizes(resnet50())
    order = list(range(len(s)))[::-1]
    b = assign_buckets(s, order, 25 * 2**20, 2**20)
    flat = [i for bk in b for i in bk]
    assert sorted(flat) == list(range(len(s)))          # every param exactly once
    assert flat == order                                  # in ready order
    assert sum(s[i] for i in b[0]) >= 2**20               # first bucket closes at >= 1 MiB
    for bk in b[1:-1]:
        tot = sum(s[i] for i in bk)
        assert tot >= 25 * 2**20 and tot - s[bk[-1]] < 25 * 2**20
    assert sum(sum(s[i] for i in bk) for bk in b) == 25557032 * 4


def test_keys_split_buckets():
    b = assign_buckets([4, 4, 4, 4], [3, 2, 1, 0], 100, 100, keys=["a", "b", "a", "b"])
    assert sorted(map(sorted, b)) == [[0, 2], [1, 3]]
