set -o pipefail
for d in 0; do
for sh in "64 256 1 1 56 512" "128 512 1 1 28 512" "256 1024 1 1 14 512"; do
  set -- $sh
  DPE_PW_DBG=$d timeout -k 10 60 python -c "
import sys, torch; sys.path.insert(0, '.')
from distributed_pytorch_example_amd.ops import ext
C = ext(); ci, co, k, s, h, B = $1, $2, $3, $4, $5, $6
xs = [torch.randn(B, h, h, ci, device='cuda').to(torch.bfloat16) for _ in range(4)]
w = (torch.randn(co, 1, 1, ci, device='cuda') / ci ** 0.5).to(torch.bfloat16)
for x in xs: C.conv_fwd(x, w, [1, 1], [0, 0], [1, 1], True, None)
torch.cuda.synchronize(); a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for r in range(10):
  for x in xs: C.conv_fwd(x, w, [1, 1], [0, 0], [1, 1], True, None)
b.record(); b.synchronize(); us = a.elapsed_time(b) * 1e3 / 40
by = B * h * h * (ci + co) * 2
print(f'dbg=$d ({ci},{co},{h}) {us:7.1f} us {by / us / 1e6:5.2f} TB/s')
" || exit 1
done
done
