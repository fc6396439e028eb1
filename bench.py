#!/usr/bin/env python3
"""Throughput benchmark -- BASELINE.json headline: ResNet-50 bf16 DDP training,
samples/sec for the whole node, one process per GPU over RCCL.

    python bench.py --gpus N --steps K --warmup W          (N=1)
    torchrun --nproc-per-node N bench.py --gpus N ...      (N>1)

Per step (all inside the timed region): forward, fused cross-entropy,
backward with bucketed RCCL all-reduce overlapped on a side stream, fused SGD
(momentum 0.9, wd 5e-5) update of fp32 masters + bf16 shadows.  Synthetic,
device-resident ImageNet-shaped batches (NCHW fp32 3x224x224, several distinct
batches cycled; the model packs them into its stem layout inside the step), random-init
weights.  Weak scaling: --batch-size images per GPU (default 512, the per-GPU
batch BASELINE.json names for ResNet-50 (config 5); measured on one MI355X:
256 -> 9.2k, 512 -> 10.0k, 1024 -> 10.7k img/s; stock PyTorch-ROCm 6.3k / 6.7k
at 256 / 512).
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# RCCL / CUDA-tensor sharing across processes needs dmabuf IPC on this driver
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "samples/sec (whole node) + DDP scaling eff., ResNet-50 bf16 at 1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "gpt2", "simplenet"])
    ap.add_argument("--batch-size", type=int, default=None,
                    help="per-GPU batch (resnet50: 512 = BASELINE config 5's per-GPU batch, sized for 288 GB HBM; "
                         "gpt2: 8 seqs)")
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--bucket-mb", type=float, default=None,
                    help="bucket cap (default: the 7-link xGMI policy of parallel/buckets.py)")
    ap.add_argument("--first-bucket-mb", type=float, default=None)
    ap.add_argument("--last-bucket-mb", type=float, default=None,
                    help="re-split the last-ready bucket (the all-reduce that cannot overlap backward) into <= this "
                         "(default: policy, 2 MiB; 0: off)")
    ap.add_argument("--comm-max-channels", type=int, default=None,
                    help="cap RCCL's channels (CUs a collective occupies while overlapping backward)")
    ap.add_argument("--grad-accum", type=int, default=1)
    ap.add_argument("--optimizer", default=None)
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--bucket-timing", type=int, default=None,
                    help="1: after the timed steps, one instrumented (untimed) step: per-bucket all-reduce time and "
                         "its overlap with backward (HIP events on the RCCL stream), reported under 'buckets' "
                         "(default: on at world size > 1, so a multi-GPU run documents its communication)")
    ap.add_argument("--force-comm", action="store_true",
                    help="run the RCCL bucket all-reduces even at world size 1 (reducer/overlap mechanics check)")
    ap.add_argument("--nbatches", type=int, default=4, help="distinct synthetic batches cycled")
    ap.add_argument("--graph", type=int, default=0,
                    help="1: capture one whole training step (forward, backward, reducer, optimizer) in a HIP graph "
                         "after the warm-up and replay it; each step copies its batch into the graph's input "
                         "buffers (world 1, grad-accum 1; dropout masks, seeded from a host counter, are "
                         "frozen at capture -- SimpleNet's)")
    ap.add_argument("--overlap-optimizer", type=int, default=0,
                    help="1: the fused optimizer steps each gradient bucket during backward on its own stream "
                         "(DDP.overlap_optimizer) instead of after it")
    ap.add_argument("--dtype", default=None, choices=[None, "fp32", "bf16"],
                    help="simplenet compute dtype (default fp32, the reference's); resnet50/gpt2 are bf16")
    return ap.parse_args()


def main():
    args = parse()
    from distributed_pytorch_example_amd.utils.env import ensure_single_process_env
    from distributed_pytorch_example_amd.parallel import dist as pdist
    from distributed_pytorch_example_amd.parallel import DDP
    from distributed_pytorch_example_amd.models import get_model
    from distributed_pytorch_example_amd.optim import build_optimizer
    from distributed_pytorch_example_amd.ops import functional as Fx

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # a bare `python bench.py --gpus N` would silently measure one GPU: refuse instead
        raise SystemExit(f"[bench] --gpus {args.gpus} needs one process per GPU: launch with "
                         f"`python -m torch.distributed.run --nproc-per-node {args.gpus} bench.py --gpus {args.gpus} ...`")
    ensure_single_process_env()
    rank, world, local_rank = pdist.init_process_group("auto", comm_max_channels=args.comm_max_channels)
    if world != args.gpus:
        raise SystemExit(f"[bench] --gpus {args.gpus} but the launcher started WORLD_SIZE={world} processes")
    dev = torch.device("cuda", local_rank) if torch.cuda.is_available() else torch.device("cpu")
    torch.manual_seed(1234 + rank)

    if args.model == "resnet50":
        bs = args.batch_size or 512
        model = get_model("resnet50").to(dev)
        opt_name, lr = args.optimizer or "sgd", args.lr or 0.1
        wd = 5e-5
        g = torch.Generator(device=dev)
        g.manual_seed(99 + rank)
        # device-resident NCHW fp32 batches (a normalising loader's output): the model's packing into the
        # stem's space-to-depth bf16 layout runs inside every timed step, as a real input would
        xs = [torch.randn(bs, 3, 224, 224, generator=g, device=dev) for _ in range(args.nbatches)]
        ys = [torch.randint(0, 1000, (bs,), device=dev, generator=g) for _ in range(args.nbatches)]
        samples_per_step = bs * args.grad_accum
        unit_mult = 1
        cfg = {"model": "resnet50-v1.5", "global_batch": bs * world * args.grad_accum, "seq_len": None,
               "image": [3, 224, 224], "per_gpu_batch": bs, "grad_accum": args.grad_accum,
               "bucket_mb": args.bucket_mb, "parallelism": f"dp{world}", "optimizer": "sgd-momentum0.9"}
        metric, unit = METRIC, "samples/s"
        num_classes = 1000
    elif args.model == "gpt2":
        bs = args.batch_size or 8
        model = get_model("gpt2").to(dev)
        opt_name, lr = args.optimizer or "adamw", args.lr or 6e-4
        wd = 0.1
        g = torch.Generator(device=dev)
        g.manual_seed(99 + rank)
        V = 50257
        toks = [torch.randint(0, V, (bs, args.seq_len + 1), device=dev, generator=g) for _ in range(args.nbatches)]
        xs = [t[:, :-1].contiguous() for t in toks]
        ys = [t[:, 1:].contiguous() for t in toks]
        samples_per_step = bs * args.seq_len * args.grad_accum
        cfg = {"model": "gpt2-small-124M", "global_batch": bs * world * args.grad_accum, "seq_len": args.seq_len,
               "parallelism": f"dp{world}", "optimizer": "adamw"}
        metric, unit = "tokens/sec (whole node), GPT-2-small bf16", "tokens/s"
        num_classes = V
    else:
        bs = args.batch_size or 64
        sdt = args.dtype or "fp32"
        model = get_model("simplenet", compute_dtype=sdt).to(dev)
        opt_name, lr = args.optimizer or "adam", args.lr or 1e-3
        wd = 0.0
        xs = [torch.randn(bs, 784, device=dev) for _ in range(args.nbatches)]
        ys = [torch.randint(0, 10, (bs,), device=dev) for _ in range(args.nbatches)]
        samples_per_step = bs * args.grad_accum
        cfg = {"model": "simplenet-mlp", "global_batch": bs * world, "seq_len": None, "parallelism": f"dp{world}",
               "compute_dtype": sdt}
        metric, unit = "samples/sec (whole node), SimpleNet MLP", "samples/s"
        num_classes = 10

    fused_loss = args.model == "gpt2"
    ddp = DDP(model, bucket_cap_mb=args.bucket_mb, first_bucket_mb=args.first_bucket_mb, force_comm=args.force_comm,
              last_bucket_mb="auto" if args.last_bucket_mb is None else (args.last_bucket_mb or None))
    if "bucket_mb" in cfg:
        cfg["bucket_mb"] = round(ddp.bucket_cap_bytes / 2**20, 2)
    if world > 1:  # the RCCL channel cap and the compute side's CU budget while buckets are in flight
        from distributed_pytorch_example_amd.ops import ext as _ext

        cfg["rccl_max_channels"] = pdist.comm_max_channels()
    opt = build_optimizer(opt_name, model.parameters(), lr=lr, weight_decay=wd)
    if args.overlap_optimizer and dev.type == "cuda" and not args.graph:
        ddp.overlap_optimizer(opt)
        cfg["optimizer_in_backward"] = True

    def step(i):
        for a in range(args.grad_accum):
            x, y = xs[(i * args.grad_accum + a) % len(xs)], ys[(i * args.grad_accum + a) % len(ys)]
            last = a == args.grad_accum - 1
            ctx = ddp.no_sync() if not last else _null()
            with ctx:
                if fused_loss:
                    loss = ddp(x, y)  # GPT-2: fused LM head + CE (logits stay inside the op)
                else:
                    loss = Fx.cross_entropy(ddp(x), y, num_classes)
                if args.grad_accum > 1:
                    loss = loss / args.grad_accum
                loss.backward()
        opt.step()
        for p in model.parameters():
            p.grad = None  # buckets re-zeroed at next forward
        return loss

    for i in range(args.warmup):
        step(i)
    if world > 1:  # after warm-up: the adaptive CU budget decided from measured comm (parallel/ddp.py)
        cfg["cu_budget"] = ddp.settle_cu_budget()
        cfg["cu_reserve_slots"] = _ext().cu_reserve_config() if dev.type == "cuda" else 0
    if args.graph and dev.type == "cuda":
        step = _graph_step(args, world, ddp, opt, model, xs, ys, fused_loss, num_classes, Fx)
    _sync(dev)
    pdist.barrier()
    _sync(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(args.warmup + i)
    _sync(dev)
    pdist.barrier()
    _sync(dev)
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64)
    if world > 1:
        import torch.distributed as dist

        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = t.item()
    ms = 1000.0 * dt / args.steps
    value = samples_per_step * world * args.steps / dt
    extra = {}
    if args.bucket_timing if args.bucket_timing is not None else world > 1:
        # one extra (untimed) step with per-bucket HIP events on the comm stream
        ddp.enable_timing(True)
        step(args.warmup + args.steps)
        _sync(dev)
        tim = ddp.bucket_timings()
        sizes = ddp.bucket_bytes()
        rows, comm, hidden = [], 0.0, 0.0
        for b, ar_ms, rel in tim:
            # rel = start of this bucket's all-reduce relative to the end of backward (negative: overlapped)
            ov = min(max(-rel, 0.0), ar_ms)
            comm += ar_ms
            hidden += ov
            rows.append({"bucket": b, "bytes": sizes[b], "allreduce_ms": round(ar_ms, 4),
                         "start_vs_bwd_end_ms": round(rel, 4)})
        extra["buckets"] = {"count": ddp.num_buckets(), "per_bucket": rows, "comm_ms": round(comm, 4),
                            "overlap_pct": round(100.0 * hidden / comm, 1) if comm > 0 else None}
    if rank == 0:
        line = {"metric": metric, "value": round(value, 2), "unit": unit, "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
                "vs_baseline": None,
                "dtype": ("bf16" if args.model != "simplenet" else sdt) if dev.type == "cuda" else "fp32",
                "data": "synthetic (device-resident, random)",
                "config": cfg, "loss": float(loss.item())}
        line.update(extra)
        print(json.dumps(line), flush=True)
    pdist.destroy_process_group()


def _graph_step(args, world, ddp, opt, model, xs, ys, fused_loss, num_classes, Fx):
    """Capture one training step in a HIP graph (torch.cuda.graph over the HIP stream) and return a
    step function that refills the static input buffers and replays it.  Every kernel of the step is
    in the graph: the launch gaps between ~400 short kernels (GPT-2) go away.  The fused optimizers
    keep their step counters and hyper-parameters on the device, so the replayed update is the
    eager one; the DDP buckets are re-zeroed by the captured forward.  The gradients are the DDP
    bucket views, so the optimizer's device table (raw gradient pointers) is valid in every replay;
    tests/test_models_gpu.py::test_graph_replayed_step_matches_eager checks replay == eager."""
    if world != 1 or args.grad_accum != 1:
        raise SystemExit("--graph: world size 1 and --grad-accum 1 only")
    sx, sy = xs[0].clone(), ys[0].clone()

    def body():
        loss = ddp(sx, sy) if fused_loss else Fx.cross_entropy(ddp(sx), sy, num_classes)
        loss.backward()
        opt.step()
        for p in model.parameters():
            p.grad = None
        return loss

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            body()
    torch.cuda.current_stream().wait_stream(side)
    if hasattr(opt, "graph_safe"):
        opt.graph_safe = True
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        gloss = body()

    def step(i):
        sx.copy_(xs[i % len(xs)], non_blocking=True)
        sy.copy_(ys[i % len(ys)], non_blocking=True)
        g.replay()
        return gloss

    return step


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
