"""Multi-process DDP plumbing on CPU/gloo (world 2/4) and launcher behaviour:
gradient averaging, no_sync accumulation, init broadcast, buffer broadcast,
end-to-end train + resume, fail-fast fault injection."""
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(rank, world, port):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    from distributed_pytorch_example_amd.parallel import dist as pdist

    torch.set_num_threads(1)
    return pdist.init_process_group("gloo")


def _native_host(ddp, world):
    """With the extension built, gloo DDP runs the C++ Reducer (host-transport mode) at world > 1."""
    from distributed_pytorch_example_amd.ops._ext import has_ext

    if has_ext():
        assert ddp.reducer.host_mode and ddp.reducer.world == world
        assert ddp.reducer.launch_order() == list(range(ddp.num_buckets()))


def _w_grad_avg(rank, world, port, q):
    _setup(rank, world, port)
    import torch.distributed as dist

    from distributed_pytorch_example_amd.models import SimpleNet
    from distributed_pytorch_example_amd.parallel import DDP

    torch.manual_seed(100 + rank)  # different init per rank -> DDP must broadcast rank 0's
    m = SimpleNet()
    m.eval()  # no dropout: deterministic grads
    ddp = DDP(m)
    # init sync: every rank now holds rank 0's parameters
    for p in m.parameters():
        ref = p.detach().clone()
        dist.broadcast(ref, 0)
        assert torch.equal(p.detach(), ref)
    torch.manual_seed(7 + rank)
    x, y = torch.randn(8, 784), torch.randint(0, 10, (8,))
    # independent local grad for comparison
    local = [torch.autograd.grad(torch.nn.functional.cross_entropy(m(x), y), list(m.parameters()))]
    loss = torch.nn.functional.cross_entropy(ddp(x), y)
    loss.backward()
    _native_host(ddp, world)
    for g_local, p in zip(local[0], m.parameters()):
        avg = g_local.clone()
        dist.all_reduce(avg)
        avg /= world
        assert torch.allclose(p.grad, avg, atol=1e-6)
    # no_sync: two local micro-batches then a synced one == average of the sum
    for p in m.parameters():
        p.grad = None
    grads_sum = [torch.zeros_like(p) for p in m.parameters()]
    for i in range(3):
        torch.manual_seed(50 + 10 * i + rank)
        xi, yi = torch.randn(4, 784), torch.randint(0, 10, (4,))
        gi = torch.autograd.grad(torch.nn.functional.cross_entropy(m(xi), yi), list(m.parameters()))
        for a, b in zip(grads_sum, gi):
            a += b
        if i < 2:
            with ddp.no_sync():
                torch.nn.functional.cross_entropy(ddp(xi), yi).backward()
        else:
            torch.nn.functional.cross_entropy(ddp(xi), yi).backward()
    for a, p in zip(grads_sum, m.parameters()):
        dist.all_reduce(a)
        a /= world
        assert torch.allclose(p.grad, a, atol=1e-5)
    q.put(("ok", rank))
    dist.destroy_process_group()


def _w_buffers(rank, world, port, q):
    _setup(rank, world, port)
    import torch.distributed as dist

    from distributed_pytorch_example_amd.models import resnet18_like
    from distributed_pytorch_example_amd.parallel import DDP

    torch.manual_seed(rank)
    m = resnet18_like(num_classes=4)
    ddp = DDP(m, broadcast_buffers=True)
    torch.manual_seed(rank + 11)
    out = ddp(torch.randn(2, 3, 32, 32))
    out.sum().backward()
    # ranks' running stats differ after a train forward on different data
    rm = m.stem.bn.running_mean.clone()
    dist.broadcast(rm, 0)
    assert rank == 0 or not torch.equal(rm, m.stem.bn.running_mean)
    # rank 1 counts one extra batch: num_batches_tracked (int64) differs across ranks too
    if rank == 1:
        for b in m.modules():
            if getattr(b, "num_batches_tracked", None) is not None:
                b.num_batches_tracked += 1
    # forward 2 (eval: no stats update) broadcasts rank 0's buffers -- floating AND integer, like
    # stock DDP's broadcast_buffers -- before running
    m.eval()
    with torch.no_grad():
        ddp(torch.randn(2, 3, 32, 32))
    n = ni = 0
    for b in m.buffers():
        ref = b.clone()
        dist.broadcast(ref, 0)
        assert torch.equal(b, ref)
        n += 1
        ni += not b.is_floating_point()
    assert n > 0 and ni > 0
    # one flat tensor per dtype (fp32 running stats, int64 counters): one broadcast each per forward
    assert sorted(str(f.dtype) for f in ddp._flat_bufs) == ["torch.float32", "torch.int64"]
    fl = next(f for f in ddp._flat_bufs if f.dtype == torch.float32)
    assert m.stem.bn.running_mean.untyped_storage().data_ptr() == fl.untyped_storage().data_ptr()
    q.put(("ok", rank))
    dist.destroy_process_group()


def _spawn(fn, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0] * world, codes
    res = [q.get(timeout=5) for _ in range(world)]
    assert sorted(r[1] for r in res) == list(range(world))


@pytest.mark.parametrize("world", [2, 4])
def test_ddp_gradient_average_and_no_sync(world):
    _spawn(_w_grad_avg, world)


def test_ddp_buffers_broadcast():
    _spawn(_w_buffers, 2)


def _launch(args, env=None, timeout=300):
    e = dict(os.environ)
    e["PYTHONPATH"] = ROOT
    e.update(env or {})
    cmd = [sys.executable, "-m", "distributed_pytorch_example_amd.launch", "--nproc-per-node", "2",
           "--master-port", str(_port()), os.path.join(ROOT, "train.py")] + args
    return subprocess.run(cmd, env=e, capture_output=True, text=True, timeout=timeout)


def test_train_e2e_and_resume(tmp_path):
    ck = str(tmp_path / "ck")
    r = _launch(["--epochs", "1", "--num-samples", "512", "--checkpoint-dir", ck, "--backend", "gloo"])
    assert r.returncode == 0, r.stderr[-2000:]
    log = r.stdout + r.stderr
    assert "Starting distributed training with 2 processes" in log
    assert "Dataset size: 512, batches per epoch: 4" in log
    assert "Model parameters: 269,322" in log
    assert os.path.exists(os.path.join(ck, "latest_model.pt")) and os.path.exists(os.path.join(ck, "best_model.pt"))
    # resume: rank 0 reads, both ranks restart at the saved epoch (re-run semantics)
    r2 = _launch(["--epochs", "2", "--num-samples", "512", "--checkpoint-dir", ck, "--backend", "gloo", "--resume",
                  os.path.join(ck, "latest_model.pt")])
    assert r2.returncode == 0, r2.stderr[-2000:]
    log2 = r2.stdout + r2.stderr
    assert log2.count("Checkpoint loaded from") == 2      # both ranks received the state
    assert "Epoch 0 completed" in log2 and "Epoch 1 completed" in log2


def test_two_simulated_nodes(tmp_path):
    """Two launcher instances on one host as 2 nodes x 1 process (static rendezvous,
    --node-rank 0/1, OMP_NUM_THREADS=1 -- SURVEY §4.4 item 2, BASELINE.md §2's
    unpinned-OMP pitfall): both agents finish and rank 0 logs a 2-process job."""
    port = str(_port())
    e = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    procs = []
    for nr in (0, 1):
        cmd = [sys.executable, "-m", "distributed_pytorch_example_amd.launch", "--nnodes", "2", "--nproc-per-node", "1",
               "--node-rank", str(nr), "--master-addr", "127.0.0.1", "--master-port", port,
               os.path.join(ROOT, "train.py"), "--epochs", "1", "--num-samples", "256",
               "--checkpoint-dir", str(tmp_path / f"ck{nr}"), "--backend", "gloo"]
        procs.append(subprocess.Popen(cmd, env=e, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=240)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert [p.returncode for p in procs] == [0, 0], outs[0][-1500:] + outs[1][-1500:]
    assert "Starting distributed training with 2 processes" in outs[0]
    assert "[Rank 1]" in outs[1]
    assert os.path.exists(tmp_path / "ck0" / "latest_model.pt")  # only global rank 0 saves
    assert not os.path.exists(tmp_path / "ck1" / "latest_model.pt")


def test_fault_injection_fails_fast(tmp_path):
    r = _launch(["--epochs", "3", "--num-samples", "2048", "--checkpoint-dir", str(tmp_path), "--backend", "gloo"],
                env={"DPE_FAULT_INJECT": "1:0:3:kill"}, timeout=120)
    assert r.returncode == 1
    assert "rank 1 (local_rank 1): exitcode -9" in r.stderr


def test_fault_injection_exception_recorded(tmp_path):
    r = _launch(["--epochs", "1", "--num-samples", "1024", "--checkpoint-dir", str(tmp_path), "--backend", "gloo"],
                env={"DPE_FAULT_INJECT": "0:0:2:raise"}, timeout=120)
    assert r.returncode == 1
    assert "injected fault at rank 0" in r.stderr


class _TwoPath(torch.nn.Module):
    """Gradients become ready in an order unlike reverse registration order:
    `late` is registered last but used first in forward, so it is ready last."""

    def __init__(self):
        super().__init__()
        self.b = torch.nn.Linear(16, 4)
        self.a = torch.nn.Linear(16, 16)
        self.late = torch.nn.Linear(16, 16)

    def forward(self, x):
        return self.b(torch.relu(self.a(torch.relu(self.late(x)))))


def _w_rebuild_and_hooks(rank, world, port, q):
    _setup(rank, world, port)
    import torch.distributed as dist

    from distributed_pytorch_example_amd.parallel import DDP, hooks

    def local_avg(m, x, y):
        g = torch.autograd.grad(torch.nn.functional.cross_entropy(m(x), y), list(m.parameters()))
        out = []
        for t in g:
            t = t.clone()
            dist.all_reduce(t)
            out.append(t / world)
        return out

    torch.manual_seed(0)
    m = _TwoPath()
    ddp = DDP(m, bucket_cap_mb=0.0005, first_bucket_mb=0.0005, debug=True)  # ~1 param per bucket
    n0 = ddp.num_buckets()
    order0 = [list(b) for b in ddp.bucket_indices]
    for step in range(3):
        torch.manual_seed(10 * step + rank)
        x, y = torch.randn(8, 16), torch.randint(0, 4, (8,))
        ref = local_avg(m, x, y)
        for p in m.parameters():
            p.grad = None
        torch.nn.functional.cross_entropy(ddp(x), y).backward()
        _native_host(ddp, world)
        for r, p in zip(ref, m.parameters()):
            assert torch.allclose(p.grad, r, atol=1e-6)
    # rebuilt once, from the observed ready order (late.* last), identically on all ranks
    assert ddp.bucket_rebuilds == 1, ddp.bucket_rebuilds
    assert [list(b) for b in ddp.bucket_indices] != order0
    fps = [None] * world
    dist.all_gather_object(fps, ddp.layout_fingerprint())
    assert len(set(fps)) == 1
    # gradient compression (bf16 all-reduce) and a custom hook
    ddp.register_comm_hook(None, hooks.bf16_compress_hook)
    x, y = torch.randn(8, 16), torch.randint(0, 4, (8,))
    ref = local_avg(m, x, y)
    for p in m.parameters():
        p.grad = None
    torch.nn.functional.cross_entropy(ddp(x), y).backward()
    _native_host(ddp, world)  # bf16 compression on the native reducer's transport
    for r, p in zip(ref, m.parameters()):
        assert torch.allclose(p.grad, r, atol=2e-2, rtol=2e-2)
    calls = []

    def scaled_hook(state, bucket):
        calls.append(bucket.index())
        t = bucket.buffer()
        dist.all_reduce(t)
        t.mul_(state["scale"] / world)
        fut = torch.futures.Future()
        fut.set_result(t)
        return fut

    ddp.register_comm_hook({"scale": 2.0}, scaled_hook)
    ref = local_avg(m, x, y)
    for p in m.parameters():
        p.grad = None
    torch.nn.functional.cross_entropy(ddp(x), y).backward()
    assert calls == list(range(ddp.num_buckets()))
    for r, p in zip(ref, m.parameters()):
        assert torch.allclose(p.grad, 2.0 * r, atol=1e-6)
    q.put(("ok", rank))
    dist.destroy_process_group()


def test_ddp_bucket_rebuild_and_comm_hooks():
    _spawn(_w_rebuild_and_hooks, 2)


def _w_layout_mismatch(rank, world, port, q):
    _setup(rank, world, port)
    import torch.distributed as dist

    from distributed_pytorch_example_amd.models import SimpleNet
    from distributed_pytorch_example_amd.parallel import DDP

    try:
        DDP(SimpleNet(), bucket_cap_mb=0.1 if rank == 0 else 25.0, debug=True)
        q.put(("no-error", rank))
    except RuntimeError as e:
        q.put(("ok" if "layout differs" in str(e) else f"wrong: {e}", rank))
    dist.destroy_process_group()


def test_ddp_debug_detects_bucket_layout_mismatch():
    _spawn(_w_layout_mismatch, 2)


def test_train_runtime_options(tmp_path):
    """Additive runtime flags on the reference CLI: bf16 gradient compression,
    DDP desync guard, watchdog heartbeat, roctx ranges, grad accumulation."""
    r = _launch(["--epochs", "1", "--num-samples", "512", "--checkpoint-dir", str(tmp_path), "--backend", "gloo",
                 "--gradient-compression", "bf16", "--ddp-debug", "--watchdog-timeout", "120", "--roctx",
                 "--grad-accum", "2"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Epoch 0 completed" in (r.stdout + r.stderr)


def _w_dispatch_identical(rank, world, port, q):
    """Every rank plans the same GEMM kernel / tile / K split for the same shape: the dispatch is a pure
    function of the shape (no per-rank timing), so DDP replicas run identical math (reference DDP(model),
    train.py:233)."""
    _setup(rank, world, port)
    import torch.distributed as dist

    from distributed_pytorch_example_amd.ops._ext import ext, has_ext

    if not has_ext():
        q.put(("ok", rank))
        return
    C = ext()
    shapes = [(8192, 2304, 768, True, True), (8192, 768, 3072, True, True), (8192, 768, 50304, True, False),
              (2304, 768, 8192, False, False), (50304, 768, 8192, False, False), (1024, 1000, 2048, True, True)]
    mine = [C.hgemm_plan(M, N, K, ak, bk, True, 2) for M, N, K, ak, bk in shapes]
    allp = [None] * world
    dist.all_gather_object(allp, mine)
    assert all(p == allp[0] for p in allp), allp
    q.put(("ok", rank))
    dist.destroy_process_group()


def test_gemm_dispatch_identical_across_ranks():
    _spawn(_w_dispatch_identical, 2)


def _w_broadcast_state(rank, world, port, q):
    _setup(rank, world, port)
    import torch.distributed as dist

    from distributed_pytorch_example_amd.utils.checkpoint import broadcast_state

    ck = None
    if rank == 0:
        torch.manual_seed(0)
        ck = {"epoch": 3, "loss": 0.25, "model_state_dict": {"w": torch.randn(5, 7), "n": torch.tensor(4, dtype=torch.int64),
                                                          "mask": torch.arange(10) % 3 == 0,
                                                          "z": torch.complex(torch.arange(4.0), -torch.arange(4.0)),
                                                          "u16": torch.arange(6).to(torch.uint16)},
              "optimizer_state_dict": {"state": {0: {"step": torch.tensor(12.0), "exp_avg": torch.randn(5, 7)}},
                                       "param_groups": [{"lr": 1e-3, "betas": (0.9, 0.999), "params": [0]}]}}
    out = broadcast_state(ck, torch.device("cpu"))
    mine = [out["model_state_dict"]["w"], out["optimizer_state_dict"]["state"][0]["exp_avg"]]
    for t in mine:
        ref = t.clone()
        dist.broadcast(ref, 0)
        assert torch.equal(t, ref)
    assert out["epoch"] == 3 and out["optimizer_state_dict"]["param_groups"][0]["betas"] == (0.9, 0.999)
    st = out["optimizer_state_dict"]["state"][0]["step"]
    assert st.dim() == 0 and float(st) == 12.0 and out["model_state_dict"]["n"].dtype == torch.int64
    # dtypes outside RCCL's set travel as byte views and come back with their dtype and values
    msd = out["model_state_dict"]
    assert msd["mask"].dtype == torch.bool and torch.equal(msd["mask"], torch.arange(10) % 3 == 0)
    assert msd["z"].dtype == torch.complex64 and torch.equal(msd["z"], torch.complex(torch.arange(4.0), -torch.arange(4.0)))
    assert msd["u16"].dtype == torch.uint16 and torch.equal(msd["u16"].to(torch.int64), torch.arange(6))
    q.put(("ok", rank))
    dist.destroy_process_group()


def test_resume_state_broadcast_as_flat_tensors():
    _spawn(_w_broadcast_state, 2)
