import sys, math, torch
sys.path.insert(0, '.')
from distributed_pytorch_example_amd.ops import ext
C = ext(); dev = 'cuda'
torch.manual_seed(0)
bf = lambda t: t.to(torch.bfloat16)
for (N, H, W, Ci, Co) in [(32, 64, 64, 256, 64), (64, 28, 28, 512, 128)]:
    a2 = bf(torch.randn(N, H, W, Co, device=dev)); w3 = bf(torch.randn(Ci, 1, 1, Co, device=dev) / math.sqrt(Co))
    outs = [C.conv_fwd(a2, w3, [1, 1], [0, 0], [1, 1], True, None) for _ in range(3)]
    C.set_pw_stream(False); ref = C.conv_fwd(a2, w3, [1, 1], [0, 0], [1, 1], True, None); C.set_pw_stream(True)
    for y, st in outs:
        print((N, H, W, Ci, Co), 'y==ref', torch.equal(y, ref[0]), 'y==y0', torch.equal(y, outs[0][0]),
              'stats rel vs ref %.2e' % ((st.sum(-1) - ref[1].sum(-1)).norm() / ref[1].sum(-1).norm()).item(),
              'stats bitwise vs run0', torch.equal(st.sum(-1), outs[0][1].sum(-1)))
