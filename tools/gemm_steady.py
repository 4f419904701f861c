"""Steady-state GEMM throughput (large shapes, tail negligible) per forced tile config (GPU only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splatformer_amd import ptv3_ops as ops  # noqa: E402

dev = torch.device("cuda")
for M, N, K in [(65536, 4096, 1024), (262144, 256, 1024), (262144, 256, 256), (262144, 128, 128), (262144, 64, 64)]:
    x = torch.randn(M, K, device=dev)
    w = torch.randn(N, K, device=dev)
    out = torch.empty(M, N, device=dev)
    for _ in range(3):
        ops.linear(x, w, out=out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(10):
        ops.linear(x, w, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"cfg={os.environ.get('SFX_GEMM_CFG', '-1')} M={M} N={N} K={K}: {ms * 1e3:.1f} us "
          f"{2 * M * N * K / ms / 1e9:.1f} TF/s", flush=True)
