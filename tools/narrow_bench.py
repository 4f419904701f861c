"""Dense K <= 128 linears of the config-B refine, timed alone (HIP events, median of 30) -- run once with
SFX_GEMM_NARROW=1 (gemm_narrow.hip) and once with 0 (gemm_kernel).  qkv shapes (N = 3K) publish max |Y| like
the refine's qkv; N == K shapes add a residual like proj.  usage: python tools/narrow_bench.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splatformer_amd import _lib  # noqa: E402
from splatformer_amd import ptv3_ops as ops  # noqa: E402

SHAPES = [(100000, 192, 64), (100000, 64, 64), (100000, 96, 64), (100000, 288, 96), (100000, 96, 96),
          (90434, 288, 96), (90434, 96, 96), (90434, 128, 96), (70349, 384, 128), (70349, 128, 128),
          (70349, 96, 128), (70349, 256, 128)]


def main():
    _lib.load()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    tag = os.environ.get("SFX_GEMM_NARROW", "1")
    for M, N, K in SHAPES:
        x = torch.randn(M, K, generator=g).to(dev)
        w = (torch.randn(N, K, generator=g) / K ** 0.5).to(dev)
        b = torch.randn(N, generator=g).to(dev)
        r = torch.randn(M, N, generator=g).to(dev) if N == K else None
        qkv = N == 3 * K
        fn = lambda: ops.linear(x, w, b, residual=r, y_amax=qkv)
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(30):
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            e.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(e) * 1e3)
        us = statistics.median(ts)
        byt = 4 * (M * K + M * N * (2 if r is not None else 1))
        print(f"narrow={tag} M={M:6d} N={N:4d} K={K:4d}: {us:7.1f} us  {byt / us / 1e3:6.0f} GB/s  "
              f"{2 * M * N * K / us / 1e6:6.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
