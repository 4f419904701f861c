"""Time a fixed list of (M, N, K) GEMM shapes (plain linear and SubM conv pair launches) with the current
SFX_GEMM_* environment; one line per shape.  GPU only: SFX_GEMM_CFG=5 python tools/gemm_sweep.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splatformer_amd import ptv3_ops as ops  # noqa: E402

SHAPES = [(37759, 256, 256), (37759, 1024, 256), (37759, 256, 1024), (37759, 768, 256), (14764, 2048, 512),
          (14764, 512, 2048), (14764, 1536, 512), (70349, 512, 128), (70349, 128, 512), (90434, 384, 96),
          (100000, 768, 128), (37759, 6912, 256)]


def main():
    dev = torch.device("cuda")
    if os.environ.get("SWEEP_CACHE_SPLIT") == "1":  # time the GEMM alone: split each A once
        cache = {}
        orig = ops.split_operand

        def cached(x):
            k = (x.data_ptr(), tuple(x.shape))
            if k not in cache:
                cache[k] = orig(x)
            return cache[k]
        ops.split_operand = cached
    tag = os.environ.get("SFX_GEMM_CFG", "auto") + "/" + os.environ.get("SFX_GEMM_PREC", "split") + \
        ("/cached" if os.environ.get("SWEEP_CACHE_SPLIT") == "1" else "")
    for M, N, K in SHAPES:
        x = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) / K ** 0.5
        b = torch.randn(N, device=dev)
        out = torch.empty(M, N, device=dev)
        for _ in range(3):
            ops.linear(x, w, b, out=out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            ops.linear(x, w, b, out=out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        ref = torch.addmm(b.double(), x.double(), w.double().T)
        err = float((out.double() - ref).norm() / ref.norm())
        print(f"{tag:12s} M={M:6d} N={N:5d} K={K:5d} {ms * 1e3:8.1f} us {2 * M * N * K / ms / 1e9:6.1f} TF/s "
              f"err {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
