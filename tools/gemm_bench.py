"""Microbenchmark of sfx_linear on the PTv3 shapes (config B stages) vs torch.matmul (hipBLASLt fp32).

python tools/gemm_bench.py  -> one line per shape: us/call and TFLOP/s for both (GPU only).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splatformer_amd import ptv3_ops as ops  # noqa: E402

SHAPES = []
for M, C in [(100000, 64), (100000, 96), (90434, 96), (70349, 128), (37759, 256), (14764, 512)]:
    SHAPES += [(M, C, C), (M, 3 * C, C), (M, 4 * C, C), (M, C, 4 * C)]
SHAPES += [(100000, 768, 120)]


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device("cuda")
    torch.backends.cuda.matmul.allow_tf32 = False
    tot_s, tot_t = 0.0, 0.0
    for M, N, K in SHAPES:
        x = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) / K ** 0.5
        b = torch.randn(N, device=dev)
        out = torch.empty(M, N, device=dev)
        us = timeit(lambda: ops.linear(x, w, b, out=out))
        ut = timeit(lambda: torch.addmm(b, x, w.t()))
        fl = 2.0 * M * N * K
        ref = torch.addmm(b, x, w.t())
        err = float((out - ref).abs().max() / ref.abs().max())
        tot_s += us
        tot_t += ut
        print(f"M={M:6d} N={N:5d} K={K:5d}  sfx {us:8.1f} us {fl / us / 1e6:6.1f} TF/s   torch {ut:8.1f} us "
              f"{fl / ut / 1e6:6.1f} TF/s  relerr {err:.1e}", flush=True)
    print(f"total sfx {tot_s / 1e3:.2f} ms  torch {tot_t / 1e3:.2f} ms")


if __name__ == "__main__":
    main()
