"""Run one window-attention shape repeatedly (for rocprofv3 counters / timing).  GPU only.
python tools/attn_one.py N C heads [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splatformer_amd import ptv3_ops as ops  # noqa: E402

n, C, H = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (37759, 256, 16)
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
dev = torch.device("cuda")
qkv = torch.randn(n, 3 * C, device=dev)
order = (torch.arange(n, device=dev) if os.environ.get("ATTN_ORDER") == "identity" else torch.randperm(n, device=dev)).int()
K = min(n, 128)
tab = ops.window_table([n], K)
win = torch.tensor(tab, dtype=torch.int32, device=dev)
out = torch.empty(n, C, device=dev)
for _ in range(3):
    ops.window_attention(qkv, order, win, len(tab), K, H, C, out=out)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
e0.record()
for _ in range(reps):
    ops.window_attention(qkv, order, win, len(tab), K, H, C, out=out)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
fl = 4.0 * K * C * n
print(f"attn N={n} C={C} H={H}: {ms * 1e3:.1f} us  {fl / ms / 1e9:.1f} TF/s (algorithmic QK^T+PV)")
