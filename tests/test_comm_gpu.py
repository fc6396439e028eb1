"""Native RCCL communicator + C++ reducer on the device.  A 1-GPU box can only
host a world of 1, so the reducer runs in `force` mode (collectives issued
even at world 1; ncclAvg over one rank is the identity): this exercises the
real comm stream, events, bucket ordering and finalize on hardware."""
import contextlib
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(scope="module")
def comm(C):
    return C.Communicator(C.rccl_unique_id(), 0, 1, 0)


def test_collectives_world1(C, comm):
    x = torch.randn(1000, device=dev)
    y = x.clone()
    comm.all_reduce(y, "sum")
    assert torch.equal(x, y)
    comm.all_reduce(y, "avg")
    assert torch.allclose(x, y)
    comm.broadcast(y, 0)
    out = torch.empty(1000, device=dev)
    comm.all_gather(x, out)
    assert torch.equal(out, x)
    comm.reduce_scatter(x, out, "sum")
    assert torch.equal(out, x)
    comm.all_to_all(x, out)
    assert torch.equal(out, x)
    b = torch.randn(77, device=dev).to(torch.bfloat16)
    comm.all_reduce(b, "max")
    comm.barrier()
    assert comm.async_error() == ""
    assert C.rccl_version() >= 22600


def test_reducer_order_and_grads(C, comm):
    from distributed_pytorch_example_amd.models import resnet18_like
    from distributed_pytorch_example_amd.ops import functional as Fx
    from distributed_pytorch_example_amd.parallel import DDP

    torch.manual_seed(0)
    m1 = resnet18_like(num_classes=10).to(dev)
    m2 = copy.deepcopy(m1)
    ddp = DDP(m2, comm=comm, force_comm=True, bucket_cap_mb=1, first_bucket_mb=0.25, timing=True)
    assert ddp.num_buckets() > 3
    x = torch.randn(8, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (8,), device=dev)
    Fx.cross_entropy(m1(x), y).backward()
    Fx.cross_entropy(ddp(x), y).backward()
    torch.cuda.synchronize()
    order = ddp.reducer.launch_order()
    assert order == list(range(ddp.num_buckets()))  # in index order, all issued
    for (n, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        assert ((a.grad - b.grad).norm() / (a.grad.norm() + 1e-12)).item() < 2e-2, n
    t = ddp.bucket_timings()
    assert len(t) == ddp.num_buckets() and all(ms >= 0 for _, ms, _ in t)
    # a second step reuses the buckets (grads re-zeroed on set_to_none)
    for p in m2.parameters():
        p.grad = None
    Fx.cross_entropy(ddp(x), y).backward()
    torch.cuda.synchronize()
    assert ddp.bucket_rebuilds == 1  # rebuilt from the observed ready order before this step
    assert ddp.reducer.launch_order() == list(range(ddp.num_buckets()))


def test_ddp_no_sync_world1(C, comm):
    from distributed_pytorch_example_amd.models import SimpleNet
    from distributed_pytorch_example_amd.ops import functional as Fx
    from distributed_pytorch_example_amd.parallel import DDP

    torch.manual_seed(1)
    m = SimpleNet().to(dev).eval()
    ddp = DDP(m, comm=comm, force_comm=True)
    x = torch.randn(16, 784, device=dev)
    y = torch.randint(0, 10, (16,), device=dev)
    with ddp.no_sync():
        Fx.cross_entropy(ddp(x), y).backward()
    g1 = [p.grad.clone() for p in m.parameters()]
    Fx.cross_entropy(ddp(x), y).backward()
    for a, p in zip(g1, m.parameters()):
        assert torch.allclose(p.grad, 2 * a, rtol=2e-2, atol=1e-4)


def test_reducer_bf16_compression_and_sync_debug(C, comm):
    """Native reducer: bf16 all-reduce of fp32 buckets (cast on the comm stream) and the
    per-bucket stream-sync debug mode; grads match the uncompressed ones to bf16 precision."""
    from distributed_pytorch_example_amd.models import resnet18_like
    from distributed_pytorch_example_amd.ops import functional as Fx
    from distributed_pytorch_example_amd.parallel import DDP

    torch.manual_seed(3)
    m1 = resnet18_like(num_classes=10).to(dev)
    m2 = copy.deepcopy(m1)
    ddp = DDP(m2, comm=comm, force_comm=True, bucket_cap_mb=2, gradient_compression="bf16", debug=True)
    x = torch.randn(8, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (8,), device=dev)
    Fx.cross_entropy(m1(x), y).backward()
    Fx.cross_entropy(ddp(x), y).backward()
    torch.cuda.synchronize()
    assert comm.async_error() == ""
    for (n, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        assert ((a.grad - b.grad).norm() / (a.grad.norm() + 1e-12)).item() < 3e-2, n


def test_wgrad_side_stream_joined_before_main_stream_reads(C):
    """Weight grads run on the side stream (bucket views, world 1, no collectives): the end-of-
    backward join must order them before main-stream work -- grads are read by a main-stream
    clone BEFORE any device synchronisation."""
    from distributed_pytorch_example_amd.models import resnet18_like
    from distributed_pytorch_example_amd.ops import _state
    from distributed_pytorch_example_amd.ops import functional as Fx
    from distributed_pytorch_example_amd.parallel import DDP

    prev = _state.set_wgrad_stream(True)
    try:
        _check_wgrad_side_stream(resnet18_like, _state, Fx, DDP)
    finally:
        _state.set_wgrad_stream(prev)


def _check_wgrad_side_stream(resnet18_like, _state, Fx, DDP):
    torch.manual_seed(5)
    m1 = resnet18_like(num_classes=10).to(dev)
    m2 = copy.deepcopy(m1)
    ddp = DDP(m2, bucket_cap_mb=4)
    x = torch.randn(64, 3, 64, 64, device=dev)
    y = torch.randint(0, 10, (64,), device=dev)
    Fx.cross_entropy(m1(x), y).backward()
    for _ in range(2):  # second step: rebuilt buckets
        for p in m2.parameters():
            p.grad = None
        Fx.cross_entropy(ddp(x), y).backward()
        early = [p.grad.clone() for p in m2.parameters()]  # main stream, no sync in between
        torch.cuda.synchronize()
        assert _state._aux_streams, "side stream was not used"
        for (n, a), b in zip(m1.named_parameters(), early):
            assert ((a.grad - b).norm() / (a.grad.norm() + 1e-12)).item() < 2e-2, n


def test_bucket_registration_world1(C, comm):
    """ncclCommRegister of the flat buckets: the reducer registers them at
    (re)build and deregisters before release; gradients are unchanged with registration on."""
    from distributed_pytorch_example_amd.models import resnet18_like
    from distributed_pytorch_example_amd.ops import functional as Fx
    from distributed_pytorch_example_amd.parallel import DDP

    t = torch.zeros(1 << 20, device=dev)
    h = comm.register_buffer(t)
    comm.deregister_buffer(h)  # 0 (declined) is a no-op as well
    torch.manual_seed(4)
    m1 = resnet18_like(num_classes=10).to(dev)
    m2 = copy.deepcopy(m1)
    ddp = DDP(m2, comm=comm, force_comm=True, bucket_cap_mb=2, register_buckets=True)
    assert 0 <= ddp.reducer.registered_buffers <= ddp.num_buckets()
    x = torch.randn(8, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (8,), device=dev)
    Fx.cross_entropy(m1(x), y).backward()
    for _ in range(2):  # second step: rebuilt (re-registered) buckets
        for p in m2.parameters():
            p.grad = None
        Fx.cross_entropy(ddp(x), y).backward()
    torch.cuda.synchronize()
    assert comm.async_error() == ""
    for (n, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        assert ((a.grad - b.grad).norm() / (a.grad.norm() + 1e-12)).item() < 2e-2, n
    print(f"registered {ddp.reducer.registered_buffers}/{ddp.num_buckets()} buckets")


def test_gpt2_fresh_gradients_equal_zeroed(C):
    """DDP leaves the GPT-2 Linear and tied-embedding gradients out of the bucket re-zero after
    zero_grad(set_to_none=True): their first backward writer overwrites (ops/_state.py grad_fresh).
    Gradients over several steps -- including a 2-micro-step no_sync accumulation and a step where
    the buckets still hold the previous step's values -- are bitwise those of the same run with
    every gradient zeroed (the tied embedding's to its scatter-add's atomic-order noise)."""
    from distributed_pytorch_example_amd.models import get_model
    from distributed_pytorch_example_amd.parallel import DDP

    torch.manual_seed(6)
    base = get_model("gpt2", n_layer=2).to(dev)
    idx = [torch.randint(0, 50257, (2, 256), device=dev) for _ in range(3)]
    tgt = [torch.randint(0, 50257, (2, 256), device=dev) for _ in range(3)]

    def run(fresh_ok):
        m = copy.deepcopy(base)
        for p in m.parameters():
            if getattr(p, "_dpe_overwrite_ok", False):
                p._dpe_overwrite_ok = fresh_ok
        ddp = DDP(m, bucket_cap_mb=8)
        out = []
        for step in range(3):
            for p in m.parameters():
                p.grad = None
            micro = 2 if step == 1 else 1
            for a in range(micro):
                ctx = ddp.no_sync() if a + 1 < micro else contextlib.nullcontext()
                with ctx:
                    ddp(idx[(step + a) % 3], tgt[(step + a) % 3]).backward()
            torch.cuda.synchronize()
            out.append([p.grad.clone() for p in m.parameters()])
        return out

    ref, got = run(False), run(True)
    assert any(getattr(p, "_dpe_overwrite_ok", False) for p in base.parameters())
    names = [n for n, _ in base.named_parameters()]
    for s, (a, b) in enumerate(zip(ref, got)):
        for n, x, y in zip(names, a, b):
            if n in ("wte", "wpe"):  # the embedding scatter-add uses float atomics: run-to-run last bits
                assert ((x - y).norm() / x.norm()).item() < 1e-6, (s, n)
            else:
                assert torch.equal(x, y), (s, n)


def test_gpt2_fresh_gradients_with_foreign_writer(C):
    """a stock-torch writer of an overwrite-tagged parameter (an auxiliary loss on the tied
    embedding, through autograd's AccumulateGrad) must not add into last step's stale bucket values:
    DDP's tensor hook zeroes a still-fresh view before the accumulation.  Gradients equal the run
    with every bucket zeroed (to the embedding scatter-add's atomic-order noise)."""
    from distributed_pytorch_example_amd.models import get_model
    from distributed_pytorch_example_amd.parallel import DDP

    torch.manual_seed(7)
    base = get_model("gpt2", n_layer=1).to(dev)
    idx = [torch.randint(0, 50257, (2, 128), device=dev) for _ in range(3)]
    tgt = [torch.randint(0, 50257, (2, 128), device=dev) for _ in range(3)]

    def run(fresh_ok):
        m = copy.deepcopy(base)
        for p in m.parameters():
            if getattr(p, "_dpe_overwrite_ok", False):
                p._dpe_overwrite_ok = fresh_ok
        ddp = DDP(m, bucket_cap_mb=8)
        out = []
        for step in range(3):
            for p in m.parameters():
                p.grad = None
            loss = ddp(idx[step], tgt[step]) + 1e-3 * (m.wte.float() ** 2).sum()  # foreign writer of wte
            loss.backward()
            torch.cuda.synchronize()
            out.append([p.grad.clone() for p in m.parameters()])
        return out

    ref, got = run(False), run(True)
    names = [n for n, _ in base.named_parameters()]
    for s, (a, b) in enumerate(zip(ref, got)):
        for n, x, y in zip(names, a, b):
            assert ((x - y).norm() / (x.norm() + 1e-12)).item() < 1e-6, (s, n)
