"""Eval-path SubM CPE on the config-B stage geometries: the register-summed fused kernel (sfx_subm_cpe_ln, with its
per-conv row-exponent pass) against the offset-major pair GEMM + pair-sum LayerNorm, per stage (HIP events, median
of 20), plus the map's row-order build and the active (16-point group, offset) fraction of the fused kernel.
usage: python tools/subm_bench.py [--only C] [--n POINTS]"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splatformer_amd import _lib  # noqa: E402
from splatformer_amd import ptv3_ops as ops  # noqa: E402
from splatformer_amd.scenes import make_scene  # noqa: E402

# (stage, cumulative pooling shift, channel counts of the Blocks on that map) -- ptv3_base, stride (1, 2, 2, 2)
STAGES = [(0, None, (64, 96)), (1, 0, (96,)), (2, 1, (128,)), (3, 2, (256,)), (4, 3, (512,))]


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", type=int, default=None)
    ap.add_argument("--n", type=int, default=100000)
    args = ap.parse_args()
    _lib.load()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    grid0 = torch.floor(make_scene(args.n, 1, seed=0)["means"] * 384).long()
    for s, shift, chans in STAGES:
        grid = grid0 if shift is None else torch.unique(grid0 >> shift, dim=0)
        n = grid.shape[0]
        smap = ops.subm_neighbors(grid.int().to(dev), None)
        t_order = timeit(lambda: (setattr(smap, "_order", None), smap.order))
        act = (smap.nbr[smap.order.long()] >= 0).cpu()
        npairs = int(act.sum()) - n
        m = n // 16 * 16
        grp = act[:m].view(-1, 16, 27).any(1)
        waste = float(grp.sum()) * 16 / (n + npairs)
        print(f"stage {s}: n={n} pairs/pt={npairs / n:.2f} order build {t_order:.1f} us, fused rows computed / "
              f"(n + pairs) = {waste:.3f}", flush=True)
        for C in chans:
            if args.only and C != args.only:
                continue
            x = torch.randn(n, C, generator=g).to(dev)
            wf = (torch.randn(C, 27 * C, generator=g) * 0.05).to(dev)
            bf, ga, be, g1, b1 = [torch.randn(C, generator=g).to(dev) for _ in range(5)]
            fl = 2.0 * (n + npairs) * C * C
            line = f"  C={C:3d}:"
            if ops.subm_fused_ok(C):
                wpk, winv = ops.subm_cpe_pack(wf)
                tr = timeit(lambda: ops.subm_rowexp(x))
                tf = timeit(lambda: ops.subm_cpe_ln(x, x, smap, wpk, winv, bf, ga, be, g1, b1, 1e-5))
                line += (f" fused {tf:7.1f} us (rowexp {tr:5.1f}; {fl / tf / 1e6:6.1f} TF/s algorithmic,"
                         f" {waste * fl / tf / 1e6:6.1f} computed)")
            w5 = wf.view(C, 3, 3, 3, C)

            def pair():
                sp = ops.subm_conv(x, smap, w5, bf, partials=ops.subm_partials_ok(x, smap, C))
                return ops.cpe_residual_ln(sp, x, ga, be, g1, b1, 1e-5)
            tp = timeit(pair)
            line += f" | pair GEMM + pair-sum LN {tp:7.1f} us ({fl / tp / 1e6:6.1f} TF/s)"
            print(line, flush=True)


if __name__ == "__main__":
    main()
