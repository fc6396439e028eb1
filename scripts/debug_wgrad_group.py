"""gpt2-tiny gradients: DDP (bucket-view grads, deferred grouped weight grads) vs a plain copy (world 1)."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29611")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
os.environ.setdefault("LOCAL_RANK", "0")
from distributed_pytorch_example_amd.models import get_model  # noqa: E402
from distributed_pytorch_example_amd.parallel import DDP  # noqa: E402
from distributed_pytorch_example_amd.parallel import dist as pdist  # noqa: E402

pdist.init_process_group("rccl")
dev = torch.device("cuda", 0)
torch.manual_seed(200)
name = sys.argv[1] if len(sys.argv) > 1 else "gpt2-tiny"
m = get_model(name).to(dev)
with torch.no_grad():
    for n, p in m.named_parameters():
        if p.dim() == 1:
            p.normal_(0, 0.05)
ref = copy.deepcopy(m)
ddp = DDP(m, bucket_cap_mb=0.25, first_bucket_mb=0.05, force_comm=True)
V, T = m.cfg.vocab_size, 64
for step in range(3):
    torch.manual_seed(31 + step)
    x = torch.randint(0, V, (4, T), device=dev)
    y = torch.randint(0, V, (4, T), device=dev)
    for p in ref.parameters():
        p.grad = None
    ref(x, y).backward()
    for p in m.parameters():
        p.grad = None
    ddp(x, y).backward()
    torch.cuda.synchronize()
    errs = sorted((((p.grad - r.grad).norm() / (r.grad.norm() + 1e-12)).item(), n)
                  for (n, p), r in zip(m.named_parameters(), ref.parameters()))[::-1]
    print(step, [(n, f"{e:.2e}") for e, n in errs[:5]], flush=True)
pdist.destroy_process_group()
