"""Locate fused-MLP mismatches: per M and C, the rows / channel blocks whose error vs the unfused path is large."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splatformer_amd import _lib  # noqa: E402
from splatformer_amd import ptv3_ops as ops  # noqa: E402


def main():
    _lib.load()
    dev = torch.device("cuda:0")
    for C in (96, 64, 128):
        for M in (4097, 20000, 100000):
            torch.manual_seed(0)
            ln = torch.nn.LayerNorm(C).to(dev)
            fc1, fc2 = torch.nn.Linear(C, 4 * C).to(dev), torch.nn.Linear(4 * C, C).to(dev)
            x = torch.randn(M, C, device=dev)
            y = ops.block_mlp(x, ln, fc1, fc2)
            h = ops.layernorm(x, ln.weight, ln.bias, ln.eps)
            m = ops.linear(h, fc1.weight, fc1.bias, act=ops.ACT_GELU)
            y0 = ops.linear(m, fc2.weight, fc2.bias, residual=x)
            d = ((y - y0).abs() / (y0 - x).abs().max()).cpu()
            bad = d > 1e-4
            rows = bad.any(1).nonzero().flatten()
            cols = bad.any(0).nonzero().flatten()
            print(f"C={C} M={M}: rel {float((y - y0).norm() / (y0 - x).norm()):.2e}, bad rows {rows.numel()} "
                  f"(first {rows[:8].tolist()}, tiles {sorted(set((rows // 64).tolist()))[:10]}), bad cols "
                  f"{cols.tolist()[:40]}", flush=True)


if __name__ == "__main__":
    main()
