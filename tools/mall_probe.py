"""Does the pair-sum LayerNorm read its partial rows from the Infinity Cache when they fit?  Times the C = 256 SubM
pair GEMM (partial rows) and the pair-sum LayerNorm right after it at several map sizes (partial bytes below / above the
256 MB MALL), per row.  GPU only: python tools/mall_probe.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from splatformer_amd import ptv3_ops as ops  # noqa: E402


def main():
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(0)
    C = 256
    w = (torch.randn(C, 3, 3, 3, C, generator=g) * 0.02).to(dev)
    b = torch.randn(C, generator=g).to(dev)
    ga, be = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    for n in (10000, 20000, 40000, 60000, 80000):
        # points on a jittered surface-like shell: ~9 neighbours per point, as the config-B C = 256 stage
        u = torch.rand(n * 3, 3, generator=g)
        r = (n * 2.2) ** 0.5
        grid = torch.unique(torch.floor(u * torch.tensor([r, r, 3.0])).int(), dim=0)[:n]
        n = grid.shape[0]
        smap = ops.subm_neighbors(grid.to(dev), None, centre=True)
        x = torch.randn(n, C, generator=g).to(dev)
        for _ in range(2):
            sp = ops.subm_conv(x, smap, w, b, partials=True)
            xo, h = ops.cpe_residual_ln(sp, x, ga, be, ga, be, 1e-5)
        torch.cuda.synchronize()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        tc = tl = 0.0
        for _ in range(5):
            e[0].record()
            sp = ops.subm_conv(x, smap, w, b, partials=True)
            e[1].record()
            xo, h = ops.cpe_residual_ln(sp, x, ga, be, ga, be, 1e-5)
            e[2].record()
            torch.cuda.synchronize()
            tc += e[0].elapsed_time(e[1]) / 5
            tl += e[1].elapsed_time(e[2]) / 5
        pb = sp.num_pairs * C * 4 / 1e6
        print(f"n {n:6d} pairs/pt {sp.num_pairs / n:5.2f} partials {pb:7.1f} MB  conv {tc * 1e3:7.1f} us "
              f"({tc * 1e6 / n:6.3f} ns/pt)  LN {tl * 1e3:7.1f} us ({tl * 1e6 / n:6.3f} ns/pt, "
              f"{(pb + 3 * n * C * 4 / 1e6) / tl / 1e3:5.2f} TB/s)", flush=True)


if __name__ == "__main__":
    main()
