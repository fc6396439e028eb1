#!/usr/bin/env python3
"""The Gram-algebra BN3 chain (bngram.hip) at the ResNet-50 bs512 shapes, for a kernel trace
(rocprofv3 --kernel-trace --stats): bn_gram (pass + reduce), bn_gram_coef (u = W G, coef), bn_gram_bwd
(coefficients / dW, Q = W^T diag(b) W with the bias partials, the Q cast)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_pytorch_example_amd.ops._ext import ext

X = ext()
reps = int(os.environ.get("REPS", "20"))
for C, HW in [(64, 56), (128, 28), (256, 14)]:
    M, Cout = 512 * HW * HW, 4 * C
    x = torch.randn(M, C, device="cuda").bfloat16()
    coef = torch.stack([torch.ones(C, device="cuda"), 0.1 * torch.randn(C, device="cuda"), torch.zeros(C, device="cuda"),
                        torch.ones(C, device="cuda")]).float()
    w = (torch.randn(Cout, C, device="cuda") * C ** -0.5).bfloat16()
    gamma, beta = torch.ones(Cout, device="cuda"), torch.zeros(Cout, device="cuda")
    part = torch.randn(2, Cout, 256, device="cuda")
    P = torch.randn(Cout, C, device="cuda")
    dg, db, dw = torch.zeros(Cout, device="cuda"), torch.zeros(Cout, device="cuda"), torch.zeros(Cout, C, device="cuda")
    for _ in range(reps):
        G, s = X.bn_gram(x, coef)
        c3, u = X.bn_gram_coef(G, s, w, M, gamma, beta, None, None, 0.1, 1e-5)
        X.bn_gram_bwd(part, P, w, u, s, c3, gamma, M, dg, db, dw)
    torch.cuda.synchronize()
    print(f"C={C} done", flush=True)
