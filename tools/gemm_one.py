"""Run one sfx_linear shape repeatedly (for rocprofv3 counter collection)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splatformer_amd import ptv3_ops as ops  # noqa: E402

M, N, K = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (100000, 256, 64)
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
dev = torch.device("cuda")
x = torch.randn(M, K, device=dev)
w = torch.randn(N, K, device=dev)
b = torch.randn(N, device=dev)
out = torch.empty(M, N, device=dev)
for _ in range(reps):
    ops.linear(x, w, b, out=out)
torch.cuda.synchronize()
print("done", M, N, K)
