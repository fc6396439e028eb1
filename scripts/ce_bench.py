#!/usr/bin/env python3
"""Time the fused cross-entropy (loss + in-place gradient) on the GPT-2 LM-head logits: 8192 x 50304
bf16 (V = 50257), in place."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import statistics
import torch
from distributed_pytorch_example_amd.ops import ext

C = ext()
B, V, ld = 8192, 50257, 50304
zs = [(torch.randn(B, ld, device="cuda") * 3).to(torch.bfloat16) for _ in range(3)]
y = torch.randint(0, V, (B,), device="cuda")
ts = []
for i in range(24):
    z = zs[i % 3]
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    C.cross_entropy(z, y, V, 1.0, True, True, -100, True)
    b.record()
    b.synchronize()
    if i >= 4:
        ts.append(a.elapsed_time(b) * 1e3)
m = statistics.median(ts)
print(f"fused CE: {m:.1f} us  {2 * B * ld * 2 / m / 1e6:.2f} TB/s", flush=True)
