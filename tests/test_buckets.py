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


def test_last_bucket_split_into_small_pieces():
    """MI355X addition: the last-ready bucket is re-split (<= last_cap bytes each, order kept);
    earlier buckets keep c10d's semantics."""
    from distributed_pytorch_example_amd.parallel.buckets import assign_buckets

    sizes = [4 << 20] * 10 + [1 << 20] * 8          # 8 x 1 MiB params become ready last
    order = list(range(len(sizes)))
    base = assign_buckets(sizes, order, 16 << 20, 4 << 20)
    split = assign_buckets(sizes, order, 16 << 20, 4 << 20, last_cap_bytes=2 << 20)
    assert base[:-1] == split[:len(base) - 1]
    tail = split[len(base) - 1:]
    assert [i for b in tail for i in b] == base[-1]
    assert all(sum(sizes[i] for i in b) <= (2 << 20) or len(b) == 1 for b in tail) and len(tail) > 1
    # a single bucket is never split (SimpleNet: the reference's one 1,077,288-B bucket)
    assert assign_buckets([1077288], [0], 25 << 20, 1 << 20, last_cap_bytes=2 << 20) == [[0]]
