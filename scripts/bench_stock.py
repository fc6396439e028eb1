#!/usr/bin/env python3
"""Comparison arm (b) of BASELINE.md §4: *stock* PyTorch-ROCm DDP on the same
ResNet-50 v1.5 topology and synthetic data -- nn.Conv2d/BatchNorm2d (MIOpen),
nn.Linear (hipBLASLt), channels_last, bf16 autocast, torch DDP with
backend="nccl" (= RCCL), torch SGD (foreach).  Same step and timing protocol
as bench.py; prints one JSON line.  This is the bar our framework must beat.
"""
import argparse
import json
import sys
import os
import time

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


class Bottleneck(nn.Module):
    def __init__(self, inp, planes, stride, down):
        super().__init__()
        self.conv1 = nn.Conv2d(inp, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.down = nn.Sequential(nn.Conv2d(inp, planes * 4, 1, stride, bias=False), nn.BatchNorm2d(planes * 4)) if down else None

    def forward(self, x):
        idn = self.down(x) if self.down is not None else x
        h = F.relu(self.bn1(self.conv1(x)))
        h = F.relu(self.bn2(self.conv2(h)))
        return F.relu(self.bn3(self.conv3(h)) + idn)


class ResNet50(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        layers, inp = [], 64
        for i, (n, planes) in enumerate(zip((3, 4, 6, 3), (64, 128, 256, 512))):
            for j in range(n):
                layers.append(Bottleneck(inp, planes, 2 if (j == 0 and i > 0) else 1, j == 0))
                inp = planes * 4
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(2048, 1000)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.bn1(self.conv1(x))), 3, 2, 1)
        x = self.layers(x)
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


class GPT2Block(nn.Module):
    def __init__(self, d=768, h=12):
        super().__init__()
        self.h = h
        self.ln_1, self.ln_2 = nn.LayerNorm(d), nn.LayerNorm(d)
        self.c_attn, self.c_proj = nn.Linear(d, 3 * d), nn.Linear(d, d)
        self.c_fc, self.mlp_proj = nn.Linear(d, 4 * d), nn.Linear(4 * d, d)

    def forward(self, x):
        B, T, C = x.shape
        q, k, v = self.c_attn(self.ln_1(x)).view(B, T, 3, self.h, C // self.h).permute(2, 0, 3, 1, 4)
        a = F.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2).reshape(B, T, C)
        x = x + self.c_proj(a)
        return x + self.mlp_proj(F.gelu(self.c_fc(self.ln_2(x)), approximate="tanh"))


class GPT2(nn.Module):
    def __init__(self, V=50257, T=1024, d=768, L=12):
        super().__init__()
        self.wte, self.wpe = nn.Embedding(V, d), nn.Embedding(T, d)
        self.h = nn.ModuleList([GPT2Block(d) for _ in range(L)])
        self.ln_f = nn.LayerNorm(d)

    def forward(self, idx):
        x = self.wte(idx) + self.wpe(torch.arange(idx.shape[1], device=idx.device))
        for b in self.h:
            x = b(x)
        return F.linear(self.ln_f(x), self.wte.weight)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--bucket-mb", type=float, default=25.0)
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "gpt2"])
    args = ap.parse_args()
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("LOCAL_RANK", "0")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    local = int(os.environ["LOCAL_RANK"])
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", local)
    torch.backends.cudnn.benchmark = True
    if args.model == "gpt2":
        model = GPT2().to(dev)
        opt = torch.optim.AdamW(model.parameters(), lr=6e-4, weight_decay=0.1, fused=True)
        toks = [torch.randint(0, 50257, (args.batch_size, 1025), device=dev) for _ in range(4)]
        xs, ys = [t[:, :-1] for t in toks], [t[:, 1:] for t in toks]
        unit = 1024
    else:
        model = ResNet50().to(dev).to(memory_format=torch.channels_last)
        opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
        xs = [torch.randn(args.batch_size, 3, 224, 224, device=dev).to(memory_format=torch.channels_last) for _ in range(4)]
        ys = [torch.randint(0, 1000, (args.batch_size,), device=dev) for _ in range(4)]
        unit = 1
    ddp = nn.parallel.DistributedDataParallel(model, device_ids=[local], bucket_cap_mb=args.bucket_mb,
                                              gradient_as_bucket_view=True)

    def step(i):
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = ddp(xs[i % 4])
            loss = F.cross_entropy(out.float().reshape(-1, out.shape[-1]), ys[i % 4].reshape(-1))
        loss.backward()
        opt.step()
        return loss

    # MIOpen's exhaustive find (cudnn.benchmark) can run for minutes at large batch:
    # keep a heartbeat on stderr so a watchdog does not take the run for hung
    import threading

    done = threading.Event()

    def beat():
        while not done.wait(30):
            print(f"[stock] warming up (MIOpen find)... rank {rank}", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()
    for i in range(args.warmup):
        step(i)
        print(f"[stock] warmup step {i + 1}/{args.warmup}", file=sys.stderr, flush=True)
    done.set()
    torch.cuda.synchronize(); dist.barrier(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(i)
    torch.cuda.synchronize(); dist.barrier(); torch.cuda.synchronize()
    dt = torch.tensor([time.perf_counter() - t0], device=dev)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    dt = dt.item()
    if rank == 0:
        print(json.dumps({"metric": f"stock-pytorch {args.model} bf16 {'tokens' if unit > 1 else 'samples'}/s (whole node)",
                          "value": round(unit * args.batch_size * world * args.steps / dt, 2), "n_gpus": world,
                          "ms_per_step": round(1000 * dt / args.steps, 3), "per_gpu_batch": args.batch_size,
                          "loss": loss.item()}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
