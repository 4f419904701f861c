"""Debug helper: linear / linear_bwd_data vs torch (fp64) for a few shapes, repeated (GPU only).
SFX_GEMM_CFG=<i> forces a tile configuration."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splatformer_amd import ptv3_ops as ops  # noqa: E402
from splatformer_amd import train_ops as tops  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator().manual_seed(0)
worst = 0.0
for (M, N, K, dact) in [(1997, 23, 768, 2), (1997, 768, 120, 0), (3000, 128, 128, 2), (777, 96, 384, 1)]:
    dy = torch.randn(M, N, generator=g)
    w = torch.randn(N, K, generator=g) / N ** 0.5
    pre = torch.randn(M, K, generator=g)
    ref = (dy.double() @ w.double())
    if dact == 2:
        ref = ref * (pre > 0).double()
    elif dact == 1:
        x = pre.double().clone().requires_grad_()
        torch.nn.functional.gelu(x).backward(torch.ones_like(x))
        ref = ref * x.grad
    wt = tops.transpose(w.to(dev))
    for rep in range(3):
        out = tops.linear_bwd_data(dy.to(dev), wt, dact=dact, dact_pre=pre.to(dev))
        e = float((out.cpu().double() - ref).norm() / ref.norm())
        worst = max(worst, e)
        print(M, N, K, dact, rep, f"{e:.2e}", flush=True)
    x = torch.randn(M, K, generator=g)
    y = ops.linear(x.to(dev), w.to(dev))
    e = float((y.cpu().double() - x.double() @ w.double().T).norm() / (x.double() @ w.double().T).norm())
    print("fwd", M, N, K, f"{e:.2e}", flush=True)
print("worst", worst)
