"""Fused Block MLP (sfx_block_mlp) vs the unfused LayerNorm + fc1(GELU) + fc2(+residual) launches on the config-B
stage shapes: per-launch time (HIP events, median of 20) and fp32-equivalent TF/s.  usage: python tools/mlp_bench.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splatformer_amd import _lib  # noqa: E402
from splatformer_amd import ptv3_ops as ops  # noqa: E402

SHAPES = [(100000, 64), (100000, 96), (90434, 96), (70349, 128), (37759, 256)]


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def main():
    _lib.load()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    for M, C in SHAPES:
        ln = torch.nn.LayerNorm(C).to(dev)
        fc1, fc2 = torch.nn.Linear(C, 4 * C).to(dev), torch.nn.Linear(4 * C, C).to(dev)
        x = torch.randn(M, C, device=dev)
        fl = 2.0 * M * 4 * C * C * 2
        tf = timeit(lambda: ops.block_mlp(x, ln, fc1, fc2))

        def unfused():
            h = ops.layernorm(x, ln.weight, ln.bias, ln.eps)
            m = ops.linear(h, fc1.weight, fc1.bias, act=ops.ACT_GELU)
            return ops.linear(m, fc2.weight, fc2.bias, residual=x)
        tu = timeit(unfused)
        y, y0 = ops.block_mlp(x, ln, fc1, fc2), unfused()
        err = float((y - y0).norm() / (y0 - x).norm())
        print(f"M={M:6d} C={C:3d}: fused {tf:8.1f} us ({fl / tf / 1e6:6.1f} TF/s, {2 * M * C * 4 / tf / 1e3:6.0f} GB/s "
              f"X+Y) | unfused {tu:8.1f} us ({fl / tu / 1e6:6.1f} TF/s) | speedup {tu / tf:5.2f} | rel diff {err:.1e}",
              flush=True)


if __name__ == "__main__":
    main()
