"""Run one window-attention backward shape repeatedly (timing / rocprofv3 counters).  GPU only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splatformer_amd import ptv3_ops as ops  # noqa: E402
from splatformer_amd import train_ops as tops  # noqa: E402

n, C, H = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (37759, 256, 16)
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
dev = torch.device("cuda")
qkv = torch.randn(n, 3 * C, device=dev)
dout = torch.randn(n, C, device=dev)
order = torch.randperm(n, device=dev).int()
K = min(n, 128)
tab = ops.window_table([n], K)
win = torch.tensor(tab, dtype=torch.int32, device=dev)
for _ in range(2):
    tops.window_attention_bwd(qkv, order, win, len(tab), K, H, C, dout)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
e0.record()
for _ in range(reps):
    tops.window_attention_bwd(qkv, order, win, len(tab), K, H, C, dout)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
print(f"attn bwd N={n} C={C} H={H}: {ms * 1e3:.1f} us (incl. dqkv zero-fill)")
