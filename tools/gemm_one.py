"""A few dense sfx_linear launches of config-B shapes, for PMC counter passes (GPU only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splatformer_amd import ptv3_ops as ops  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
for M, N, K in [(37759, 1024, 256), (14764, 512, 2048), (70349, 512, 128)]:
    x = torch.randn(M, K, device=dev, generator=g)
    w = torch.randn(N, K, device=dev, generator=g) * K ** -0.5
    for _ in range(3):
        ops.linear(x, w, None)
torch.cuda.synchronize()
print("ok")
