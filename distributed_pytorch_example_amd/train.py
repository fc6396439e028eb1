"""Training application -- CLI-, log- and checkpoint-compatible with the
reference `train.py` (`train.py:212-318`), executed on the MI355X stack.

Same 6 flags with the same defaults (`train.py:213-221`), the same log lines
(`train.py:77-80,226-247,285-316`), the same per-epoch flow (set_epoch ->
train -> validate -> metric all-reduce / world -> rank-0 checkpoints ->
barrier) and the same checkpoint files/keys.  Additive flags select the
BASELINE-scope models, backend, bucket size, grad accumulation, etc.

Deliberate fixes: resume is read by rank 0 and broadcast; the
training loss is accumulated on the device (the reference forces a device
sync with ``loss.item()`` every step, `train.py:141`); synthetic data lives in
HBM (no DataLoader worker processes, no per-batch H2D) unless ``--loader torch``.
"""
from __future__ import annotations

import argparse
import os
import time

import torch
from torch.distributed.elastic.multiprocessing.errors import record

from .data import SyntheticDataset, SyntheticTokens, create_data_loader
from .models import get_model
from .ops import functional as Fx
from .optim import build_optimizer
from .parallel import DDP
from .parallel import dist as pdist
from .utils.checkpoint import load_checkpoint, resume_exists, save_checkpoint, wait_pending
from .utils.env import ensure_single_process_env
from .utils.logging import get_logger
from .utils import fault, tracing

logger = get_logger("__main__")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser()
    # ---- reference flags (train.py:213-221), identical names and defaults
    p.add_argument("--epochs", type=int, default=10)
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--lr", type=float, default=0.001)
    p.add_argument("--num-samples", type=int, default=10000)
    p.add_argument("--checkpoint-dir", type=str, default="./checkpoints")
    p.add_argument("--resume", type=str, default=None)
    # ---- additive
    p.add_argument("--model", default="simplenet", choices=["simplenet", "resnet50", "resnet_tiny", "gpt2", "gpt2-tiny"])
    p.add_argument("--backend", default="auto", choices=["auto", "rccl", "nccl", "gloo"])
    p.add_argument("--dtype", default=None, choices=[None, "fp32", "bf16"],
                   help="compute dtype on the GPU (default: fp32 for simplenet as the reference, bf16 otherwise; "
                        "fp32 masters and gradients always)")
    p.add_argument("--optimizer", default=None, choices=[None, "adam", "adamw", "sgd"])
    p.add_argument("--weight-decay", type=float, default=0.0)
    p.add_argument("--bucket-mb", type=float, default=None,
                   help="gradient bucket cap (default: the 7-link xGMI policy, parallel/buckets.py)")
    p.add_argument("--last-bucket-mb", type=float, default=None,
                   help="re-split the last-ready gradient bucket into pieces of at most this size (0: off; "
                        "default: policy, 2 MiB)")
    p.add_argument("--comm-max-channels", type=int, default=None,
                   help="cap RCCL's channels (= CUs a collective occupies while it overlaps backward)")
    p.add_argument("--grad-accum", type=int, default=1)
    p.add_argument("--seed", type=int, default=None, help="seed the synthetic data (reference: unseeded)")
    p.add_argument("--loader", default="auto", choices=["auto", "device", "torch"])
    p.add_argument("--image-size", type=int, default=224)
    p.add_argument("--seq-len", type=int, default=1024)
    p.add_argument("--max-steps", type=int, default=None, help="stop each epoch after this many steps")
    p.add_argument("--async-checkpoint", action="store_true")
    p.add_argument("--auto-resume", action="store_true", help="resume from <checkpoint-dir>/latest_model.pt if present")
    p.add_argument("--profile", type=str, default=None, help="write a torch.profiler chrome trace to this path")
    p.add_argument("--roctx", action="store_true", help="roctx ranges (forward/backward/optimizer) for rocprofv3")
    p.add_argument("--gradient-compression", default="none", choices=["none", "bf16"],
                   help="all-reduce bf16 copies of the fp32 gradient buckets")
    p.add_argument("--ddp-debug", action="store_true", help="cross-rank bucket-layout check + per-bucket stream sync")
    p.add_argument("--watchdog-timeout", type=float, default=None,
                   help="abort the job when no training step completes for this many seconds or RCCL reports an "
                        "async error (0 = off; default: 1800 s -- the reference's gloo collective timeout -- on the "
                        "rccl backend at world > 1, off otherwise)")
    p.add_argument("--watchdog-checkpoint-grace", type=float, default=600.0,
                   help="extra seconds the watchdog allows in the end-of-epoch barrier (rank 0 writes checkpoints)")
    return p


def _datasets(args, device):
    if args.model == "simplenet":
        tr = SyntheticDataset(args.num_samples, 784, 10, seed=args.seed)
        va = SyntheticDataset(args.num_samples // 10, 784, 10, seed=None if args.seed is None else args.seed + 1)
        return tr, va, 10
    if args.model.startswith("resnet"):
        shp = (3, args.image_size, args.image_size)
        ncls = 1000 if args.model == "resnet50" else 10
        tr = SyntheticDataset(args.num_samples, shp, ncls, seed=args.seed)
        va = SyntheticDataset(max(1, args.num_samples // 10), shp, ncls, seed=None if args.seed is None else args.seed + 1)
        return tr, va, ncls
    vocab = 50257 if args.model == "gpt2" else 512
    tr = SyntheticTokens(args.num_samples, args.seq_len, vocab, seed=args.seed)
    va = SyntheticTokens(max(1, args.num_samples // 10), args.seq_len, vocab, seed=None if args.seed is None else args.seed + 1)
    return tr, va, vocab


def train_epoch(model, loader, optimizer, criterion, device, epoch, rank, grad_accum=1, max_steps=None, watchdog=None,
                fused_loss=False):
    """Reference `train_epoch` (`train.py:119-151`); loss accumulated on device.  ``fused_loss``: the
    model takes the targets and returns the loss itself (GPT-2's fused LM head + CE, reference
    `train.py:136-137` as one op: the [B, T, V] logits never materialise)."""
    model.train()
    total_loss = torch.zeros((), dtype=torch.float64, device=device)
    num_batches = 0
    nb = len(loader)
    # the epoch's last micro-batch always syncs and steps, also when --max-steps cuts the epoch
    # short: leftover no_sync gradients must not leak into the next epoch's first update
    n_eff = min(nb, max_steps) if max_steps is not None else nb
    for batch_idx, (data, target) in enumerate(loader):
        if max_steps is not None and batch_idx >= max_steps:
            break
        fault.maybe_inject(epoch, batch_idx)
        data, target = data.to(device, non_blocking=True), target.to(device, non_blocking=True)
        sync = (batch_idx + 1) % grad_accum == 0 or batch_idx + 1 == n_eff
        ctx = model.no_sync() if (not sync and hasattr(model, "no_sync")) else _null()
        with ctx:
            with tracing.range("forward"):
                if fused_loss:
                    loss = model(data, target)
                else:
                    output = model(data)
                    loss = criterion(output, target)
            with tracing.range("backward"):
                (loss / grad_accum if grad_accum > 1 else loss).backward()
        if sync:
            with tracing.range("optimizer"):
                optimizer.step()
                optimizer.zero_grad()
        if watchdog is not None:
            watchdog.beat()
        total_loss += loss.detach()
        num_batches += 1
        if batch_idx % 10 == 0 and rank == 0:
            logger.info(f"Epoch {epoch}, Batch {batch_idx}/{nb}, Loss: {loss.item():.4f}")
    return (total_loss / max(1, num_batches)).item()


@torch.no_grad()
def validate(model, loader, criterion, device, num_classes, max_steps=None, watchdog=None):
    """Reference `validate` (`train.py:154-175`): mean of per-batch losses, accuracy in %."""
    model.eval()
    total_loss = torch.zeros((), dtype=torch.float64, device=device)
    correct = torch.zeros((), dtype=torch.float64, device=device)
    total = 0
    nbatches = 0
    for i, (data, target) in enumerate(loader):
        if max_steps is not None and i >= max_steps:
            break
        data, target = data.to(device), target.to(device)
        output = model(data)
        s, c = Fx.cross_entropy_eval(output, target, num_classes)
        total_loss += s / target.numel()
        correct += c
        total += target.numel()
        nbatches += 1
        if watchdog is not None:
            watchdog.beat()
    return (total_loss / max(1, nbatches)).item(), (100.0 * correct / max(1, total)).item()


def _dtype_kw(args) -> dict:
    """--dtype -> model kwargs: SimpleNet runs fp32 (reference) or bf16; the BASELINE-scope models are bf16."""
    if args.model == "simplenet":
        return {"compute_dtype": args.dtype or "fp32"}
    if args.dtype == "fp32":
        raise SystemExit(f"--dtype fp32 is implemented for simplenet only ({args.model} runs bf16 with fp32 masters)")
    return {}


@record
def main(argv=None):
    args = build_parser().parse_args(argv)
    ensure_single_process_env()
    rank, world_size, local_rank = pdist.init_process_group(args.backend, comm_max_channels=args.comm_max_channels)
    logger.info(f"Initialized process group: rank={rank}, world_size={world_size}, local_rank={local_rank}")
    device = pdist.get_device(local_rank)

    logger.info(f"Starting distributed training with {world_size} processes")
    logger.info(f"Configuration: epochs={args.epochs}, batch_size={args.batch_size}, lr={args.lr}")

    model = get_model(args.model, **_dtype_kw(args)).to(device)
    model = DDP(model, bucket_cap_mb=args.bucket_mb,
                last_bucket_mb="auto" if args.last_bucket_mb is None else (args.last_bucket_mb or None),
                gradient_compression=None if args.gradient_compression == "none" else args.gradient_compression,
                debug=args.ddp_debug or None)
    if args.roctx:
        tracing.enable(True)
    wd_timeout = pdist.default_watchdog_timeout(args.watchdog_timeout, pdist.backend(), world_size)
    watchdog = pdist.start_watchdog(wd_timeout) if wd_timeout > 0 else None
    logger.info(f"Model parameters: {sum(p.numel() for p in model.parameters()):,}")

    train_dataset, val_dataset, num_classes = _datasets(args, device)
    mode = args.loader if args.loader != "auto" else ("device" if device.type == "cuda" else "torch")
    train_loader, train_sampler = create_data_loader(train_dataset, args.batch_size, rank, world_size, mode=mode,
                                                     device=device)
    val_loader, _ = create_data_loader(val_dataset, args.batch_size, rank, world_size, mode=mode, device=device)
    logger.info(f"Dataset size: {len(train_dataset)}, batches per epoch: {len(train_loader)}")

    opt_name = args.optimizer or ("adam" if args.model == "simplenet" else ("sgd" if args.model.startswith("resnet") else "adamw"))
    optimizer = build_optimizer(opt_name, model.parameters(), lr=args.lr, weight_decay=args.weight_decay)

    def criterion(out, tgt):
        return Fx.cross_entropy(out, tgt, num_classes)

    start_epoch = 0
    if rank == 0:
        os.makedirs(args.checkpoint_dir, exist_ok=True)
    resume = args.resume
    if resume is None and args.auto_resume:
        resume = os.path.join(args.checkpoint_dir, "latest_model.pt")
    if resume_exists(resume):
        start_epoch = load_checkpoint(model, optimizer, resume, device)

    pdist.barrier()

    best_accuracy = 0.0
    start_time = time.time()
    prof = _profiler(args.profile, rank)

    for epoch in range(start_epoch, args.epochs):
        epoch_start = time.time()
        train_sampler.set_epoch(epoch)
        train_loss = train_epoch(model, train_loader, optimizer, criterion, device, epoch, rank, args.grad_accum,
                                 args.max_steps, watchdog, fused_loss=args.model.startswith("gpt2"))
        val_loss, val_accuracy = validate(model, val_loader, criterion, device, num_classes, args.max_steps, watchdog)

        metrics = torch.tensor([train_loss, val_loss, val_accuracy], device=device)
        pdist.all_reduce(metrics, "sum")
        metrics /= world_size
        avg_train_loss, avg_val_loss, avg_val_accuracy = (v.item() for v in metrics)

        epoch_time = time.time() - epoch_start
        if rank == 0:
            logger.info(f"Epoch {epoch} completed in {epoch_time:.2f}s")
            logger.info(f"  Train Loss: {avg_train_loss:.4f}")
            logger.info(f"  Val Loss: {avg_val_loss:.4f}, Val Accuracy: {avg_val_accuracy:.2f}%")
            nb = min(len(train_loader), args.max_steps or len(train_loader))
            logger.info(f"  Throughput: {nb * args.batch_size * world_size / epoch_time:.1f} samples/s (incl. validation)")
            # no step heartbeat while rank 0 writes (RCCL async errors are still polled)
            with (watchdog.suspended() if watchdog is not None else _null()):
                if avg_val_accuracy > best_accuracy:
                    best_accuracy = avg_val_accuracy
                    save_checkpoint(model, optimizer, epoch, avg_train_loss,
                                    os.path.join(args.checkpoint_dir, "best_model.pt"), args.async_checkpoint)
                save_checkpoint(model, optimizer, epoch, avg_train_loss,
                                os.path.join(args.checkpoint_dir, "latest_model.pt"), args.async_checkpoint)
        if prof is not None:
            prof.step()
        # the other ranks wait here for rank 0's write: stall detection stays on, with a bounded
        # extra allowance for the checkpoint (a peer dying in this barrier still aborts the job)
        with (watchdog.grace(args.watchdog_checkpoint_grace) if watchdog is not None else _null()):
            pdist.barrier()

    wait_pending()
    if watchdog is not None:
        watchdog.stop()
    total_time = time.time() - start_time
    if prof is not None:
        prof.__exit__(None, None, None)
    if rank == 0:
        logger.info(f"Training completed in {total_time:.2f}s")
        logger.info(f"Best validation accuracy: {best_accuracy:.2f}%")
    pdist.destroy_process_group()


def _profiler(path, rank):
    if not path:
        return None
    from torch.profiler import ProfilerActivity, profile

    acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if torch.cuda.is_available() else [])

    def handler(p):
        p.export_chrome_trace(path.replace(".json", f".rank{rank}.json"))

    prof = profile(activities=acts, on_trace_ready=handler)
    prof.__enter__()
    return prof


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


if __name__ == "__main__":
    main()
