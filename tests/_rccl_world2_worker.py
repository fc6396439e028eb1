"""One rank of the N-process native-reducer tests (tests/test_ddp_rccl_world2_gpu.py; N = 2 or 4).

All ranks share GPU 0; each process gets its own NCCL_HOSTID so RCCL treats them
as N hosts and connects them through its socket transport -- the C++ Reducer
then issues real world-N RCCL all-reduces (Reducer::launch with world() == N).  At
N = 4 the rank-0 bucket-order broadcast reaches three peers and RCCL runs a
multi-peer ring, which world 2 (a degenerate ring) never exercises.
"""
import copy
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_pytorch_example_amd.models import resnet18_like  # noqa: E402
from distributed_pytorch_example_amd.ops import functional as Fx  # noqa: E402
from distributed_pytorch_example_amd.parallel import DDP  # noqa: E402
from distributed_pytorch_example_amd.parallel import dist as pdist  # noqa: E402


def rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def avg_local_grads(m, x, y, world):
    """Rank-averaged plain-backward grads (the all-reduce done on the gloo control plane)."""
    for p in m.parameters():
        p.grad = None
    Fx.cross_entropy(m(x), y).backward()
    out = []
    for p in m.parameters():
        g = p.grad.detach().float().cpu()
        dist.all_reduce(g)
        out.append((g / world).to(p.device))
    return out


def main():
    rank, world, _ = pdist.init_process_group("rccl")
    dev = torch.device("cuda", 0)
    if os.environ.get("DPE_RCCL_MAX_CHANNELS"):  # channel cap applied before ncclCommInitRank
        assert pdist.comm_max_channels() == int(os.environ["DPE_RCCL_MAX_CHANNELS"])
        assert os.environ["NCCL_MAX_NCHANNELS"] == os.environ["DPE_RCCL_MAX_CHANNELS"]
    torch.manual_seed(100 + rank)  # different init per rank: DDP's init broadcast (RCCL) must align them
    m = resnet18_like(num_classes=10).to(dev)
    ref = copy.deepcopy(m)  # plain-autograd twin (copied before DDP attaches bucket views / hooks)
    ddp = DDP(m, bucket_cap_mb=1, first_bucket_mb=0.25)
    assert ddp._native and ddp.reducer.world == world, f"native RCCL reducer expected at world {world}"
    ref.load_state_dict(m.state_dict())  # rank 0's weights after the init broadcast
    for p in m.parameters():  # init sync over RCCL
        q = p.detach().float().cpu()
        dist.broadcast(q, 0)
        assert torch.equal(q.to(dev), p.detach().float())
    checks = []
    for step in range(3):  # step 1 runs on the buckets rebuilt from the observed ready order
        torch.manual_seed(7 + 10 * step + rank)
        x = torch.randn(8, 3, 32, 32, device=dev)
        y = torch.randint(0, 10, (8,), device=dev)
        want = avg_local_grads(ref, x, y, world)
        for p in m.parameters():
            p.grad = None
        Fx.cross_entropy(ddp(x), y).backward()
        torch.cuda.synchronize()
        assert ddp.reducer.launch_order() == list(range(ddp.num_buckets()))
        checks.append(max(rel(p.grad, w) for p, w in zip(m.parameters(), want)))
        if step == 1:
            layout_after_rebuild = ddp.layout_fingerprint()
    assert ddp.bucket_rebuilds == 1
    # the rebuilt layout (rank 0's observed order, broadcast) is identical on every rank
    fps = [None] * world
    dist.all_gather_object(fps, layout_after_rebuild)
    assert len(set(fps)) == 1, fps
    assert max(checks) < 1e-4, checks
    # no_sync: two local micro-steps + one synced == rank average of the summed grads
    for p in m.parameters():
        p.grad = None
    for p in ref.parameters():
        p.grad = None
    xs = []
    for i in range(3):
        torch.manual_seed(50 + i + 10 * rank)
        xs.append((torch.randn(4, 3, 32, 32, device=dev), torch.randint(0, 10, (4,), device=dev)))
    for i, (x, y) in enumerate(xs):
        Fx.cross_entropy(ref(x), y).backward()
        if i < 2:
            with ddp.no_sync():
                Fx.cross_entropy(ddp(x), y).backward()
        else:
            Fx.cross_entropy(ddp(x), y).backward()
    torch.cuda.synchronize()
    for p, r in zip(m.parameters(), ref.parameters()):
        g = r.grad.detach().float().cpu()
        dist.all_reduce(g)
        assert rel(p.grad, (g / world).to(dev)) < 1e-4
    # bf16 gradient compression on the RCCL path
    ddp.register_comm_hook(None, __import__("distributed_pytorch_example_amd.parallel.hooks",
                                            fromlist=["bf16_compress_hook"]).bf16_compress_hook)
    torch.manual_seed(99 + rank)
    x = torch.randn(8, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (8,), device=dev)
    want = avg_local_grads(ref, x, y, world)
    for p in m.parameters():
        p.grad = None
    Fx.cross_entropy(ddp(x), y).backward()
    torch.cuda.synchronize()
    assert ddp._native and max(rel(p.grad, w) for p, w in zip(m.parameters(), want)) < 2e-2
    # metric all-reduce + barrier over RCCL (reference C7 / C8)
    t = torch.tensor([float(rank + 1)], device=dev)
    pdist.all_reduce(t)
    assert t.item() == world * (world + 1) / 2
    pdist.barrier()
    assert pdist.check_health() == ""
    print(f"rank {rank} ok: world-{world} RCCL reducer, max rel err {max(checks):.2e}, "
          f"{ddp.reducer.registered_buffers}/{ddp.num_buckets()} bucket buffers ncclCommRegister'ed", flush=True)
    pdist.destroy_process_group()


def main_gpt2():
    """gpt2-tiny at world 2: the tied wte gradient is written by two kernels (LM-head weight grad and
    embedding backward, use-counted), the Linear bias grads come out of the TN weight-grad GEMM, the
    buckets are rebuilt after step 0, no_sync accumulates locally -- all against rank-averaged
    plain-backward gradients of an identical copy."""
    from distributed_pytorch_example_amd.models import get_model

    rank, world, _ = pdist.init_process_group("rccl")
    dev = torch.device("cuda", 0)
    torch.manual_seed(200 + rank)
    m = get_model("gpt2-tiny").to(dev)
    with torch.no_grad():  # non-zero biases / LN params: every gradient path carries signal
        for n, p in m.named_parameters():
            if p.dim() == 1:
                p.normal_(0, 0.05)
    ref = copy.deepcopy(m)
    ddp = DDP(m, bucket_cap_mb=0.25, first_bucket_mb=0.05)
    assert ddp._native and ddp.reducer.world == world
    ref.load_state_dict(m.state_dict())
    V, T = m.cfg.vocab_size, 64

    def batch(seed):
        torch.manual_seed(seed)
        return (torch.randint(0, V, (4, T), device=dev), torch.randint(0, V, (4, T), device=dev))

    def plain_avg(x, y):
        for p in ref.parameters():
            p.grad = None
        ref(x, y).backward()
        out = []
        for p in ref.parameters():
            g = p.grad.detach().float().cpu()
            dist.all_reduce(g)
            out.append((g / world).to(dev))
        return out

    checks = []
    for step in range(3):  # step 1 onwards: buckets rebuilt from the observed ready order
        x, y = batch(31 + 10 * step + rank)
        want = plain_avg(x, y)
        for p in m.parameters():
            p.grad = None
        ddp(x, y).backward()
        torch.cuda.synchronize()
        assert ddp.reducer.launch_order() == list(range(ddp.num_buckets()))
        errs = {n: rel(p.grad, w) for (n, p), w in zip(m.named_parameters(), want)}
        checks.append(max(errs.values()))
        assert checks[-1] < 1e-4, (step, sorted(errs.items(), key=lambda kv: -kv[1])[:4])
    assert ddp.bucket_rebuilds == 1
    # no_sync: two local micro-steps + one synced == rank average of the summed grads
    for p in list(m.parameters()) + list(ref.parameters()):
        p.grad = None
    for i in range(3):
        x, y = batch(70 + i + 10 * rank)
        ref(x, y).backward()
        if i < 2:
            with ddp.no_sync():
                ddp(x, y).backward()
        else:
            ddp(x, y).backward()
    torch.cuda.synchronize()
    for p, r in zip(m.parameters(), ref.parameters()):
        g = r.grad.detach().float().cpu()
        dist.all_reduce(g)
        assert rel(p.grad, (g / world).to(dev)) < 1e-4
    print(f"rank {rank} ok: world-{world} RCCL reducer gpt2-tiny, max rel err {max(checks):.2e}, "
          f"{ddp.num_buckets()} buckets", flush=True)
    pdist.destroy_process_group()


def main_ovopt():
    """DDP.overlap_optimizer at world N: the optimizer stream must wait for each bucket's
    RCCL all-reduce (Reducer.stream_wait_comm) -- and, on the bf16 hook path, for the cast-back on the
    comm stream -- before stepping it.  Against the same model stepped after backward: the parameters
    after 4 steps (one bucket rebuild included) agree to the model's own run-to-run noise, and every
    rank holds bitwise the same parameters (a too-early wait would step un-reduced, rank-local grads)."""
    from distributed_pytorch_example_amd.models import get_model
    from distributed_pytorch_example_amd.optim import build_optimizer
    from distributed_pytorch_example_amd.parallel.hooks import bf16_compress_hook

    rank, world, _ = pdist.init_process_group("rccl")
    dev = torch.device("cuda", 0)
    out = []
    for model, opt_name in (("resnet_tiny", "sgd"), ("gpt2_tiny", "adamw")):
        for comp in (None, "bf16"):
            torch.manual_seed(300)  # same init on every rank (the init broadcast also aligns them)
            kw = {"num_classes": 10} if model == "resnet_tiny" else {}
            base = get_model(model, **kw).to(dev)
            runs = {}
            for overlap in (False, "again", True):
                m = copy.deepcopy(base)
                ddp = DDP(m, bucket_cap_mb=0.25, first_bucket_mb=0.05)
                if comp == "bf16":
                    ddp.register_comm_hook(None, bf16_compress_hook)
                assert ddp._native and ddp.reducer.world == world
                opt = build_optimizer(opt_name, m.parameters(), lr=1e-2, weight_decay=1e-2)
                if overlap is True:
                    ddp.overlap_optimizer(opt)
                g = torch.Generator(device=dev).manual_seed(11 + rank)  # rank-local data: grads differ
                for step in range(4):
                    if model == "resnet_tiny":
                        x = torch.randn(8, 3, 32, 32, device=dev, generator=g)
                        y = torch.randint(0, 10, (8,), device=dev, generator=g)
                        loss = Fx.cross_entropy(ddp(x), y, 10)
                    else:
                        x = torch.randint(0, 512, (2, 64), device=dev, generator=g)
                        y = torch.randint(0, 512, (2, 64), device=dev, generator=g)
                        loss = ddp(x, y)
                    loss.backward()
                    opt.step()
                    for p in m.parameters():
                        p.grad = None
                torch.cuda.synchronize()
                assert ddp.num_buckets() > 2
                runs[overlap] = [p.detach().float().clone() for p in m.parameters()]
                # identical on every rank: the all-reduced gradients are the same bits everywhere
                flat = torch.cat([p.reshape(-1) for p in runs[overlap]]).cpu()
                allf = [torch.empty_like(flat) for _ in range(world)]
                dist.all_gather(allf, flat)
                assert all(torch.equal(allf[0], f) for f in allf), (model, comp, overlap, "ranks diverged")

            def dev_(x, y):
                return max(((a - b).abs().max() / (b.abs().max() + 1e-30)).item() for a, b in zip(x, y))

            noise = dev_(runs["again"], runs[False])
            d = dev_(runs[True], runs[False])
            assert d <= 10 * noise + 1e-6, (model, comp, d, noise)
            out.append(f"{model}/{comp or 'fp32'} {d:.1e} (noise {noise:.1e})")
    print(f"rank {rank} ok: world-{world} overlap_optimizer " + ", ".join(out), flush=True)
    pdist.destroy_process_group()


if __name__ == "__main__":
    mode = sys.argv[1] if len(sys.argv) > 1 else ""
    {"gpt2": main_gpt2, "ovopt": main_ovopt}.get(mode, main)()
