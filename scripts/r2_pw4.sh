set -o pipefail
for st in True False; do
for sh in "64 256 56" "128 512 28" "256 1024 14"; do
  set -- $sh
  timeout -k 10 60 python -c "
import sys, torch; sys.path.insert(0, '.')
from distributed_pytorch_example_amd.ops import ext
C = ext(); ci, co, h, B = $1, $2, $3, 512
xs = [torch.randn(B, h, h, ci, device='cuda').to(torch.bfloat16) for _ in range(4)]
w = (torch.randn(co, 1, 1, ci, device='cuda') / ci ** 0.5).to(torch.bfloat16)
for x in xs: C.conv_fwd(x, w, [1, 1], [0, 0], [1, 1], $st, None)
torch.cuda.synchronize(); a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for r in range(10):
  for x in xs: C.conv_fwd(x, w, [1, 1], [0, 0], [1, 1], $st, None)
b.record(); b.synchronize(); us = a.elapsed_time(b) * 1e3 / 40
print(f'stats=$st ({ci},{co},{h}) {us:7.1f} us {B * h * h * (ci + co) * 2 / us / 1e6:5.2f} TB/s')
" || exit 1
done
done
