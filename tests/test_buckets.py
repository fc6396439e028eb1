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
    # the last-ready 2 pieces are small, the rest of the tail stays one bucket
    assert len(tail) == 3 and all(sum(sizes[i] for i in b) <= (2 << 20) for b in tail[1:])
    assert sum(sizes[i] for i in tail[0]) > (2 << 20)
    # a single bucket is never split (SimpleNet: the reference's one 1,077,288-B bucket)
    assert assign_buckets([1077288], [0], 25 << 20, 1 << 20, last_cap_bytes=2 << 20) == [[0]]


def test_xgmi_bucket_policy():
    from distributed_pytorch_example_amd.parallel.buckets import xgmi_bucket_policy

    first, cap, last = xgmi_bucket_policy(8, 25_557_032 * 4)  # ResNet-50 fp32 grads
    assert first == 1.0 and last == 2.0 and 20 < cap < 30
    assert xgmi_bucket_policy(8, 124_439_808 * 4)[1] == 64.0  # GPT-2-small: capped at 64 MiB
    small = xgmi_bucket_policy(8, 1_077_288)[1]  # SimpleNet: the bandwidth floor (one bucket)
    assert 16 <= small < 25
    assert xgmi_bucket_policy(1, 25_557_032 * 4) == xgmi_bucket_policy(2, 25_557_032 * 4)


def test_ddp_default_buckets_follow_policy():
    import torch

    from distributed_pytorch_example_amd.parallel import DDP
    from distributed_pytorch_example_amd.parallel.buckets import xgmi_bucket_policy

    m = torch.nn.Sequential(torch.nn.Linear(64, 64), torch.nn.Linear(64, 8))
    d = DDP(m)
    nbytes = 4 * sum(p.numel() for p in m.parameters())
    assert d.bucket_cap_bytes == int(xgmi_bucket_policy(1, nbytes)[1] * 2**20)
    assert DDP(m, bucket_cap_mb=25).bucket_cap_bytes == 25 * 2**20


def test_comm_max_channels_env(tmp_path):
    import subprocess
    import sys

    code = ("import os; os.environ.update(RANK='0', WORLD_SIZE='1', LOCAL_RANK='0', MASTER_ADDR='127.0.0.1', "
            "MASTER_PORT='29733'); from distributed_pytorch_example_amd.parallel import dist as d; "
            "d.init_process_group('gloo', comm_max_channels=8); "
            "assert os.environ['NCCL_MAX_NCHANNELS'] == '8' and d.comm_max_channels() == 8; print('ok')")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       cwd=__import__("os").path.dirname(__import__("os").path.dirname(__file__)))
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]
