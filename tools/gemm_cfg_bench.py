"""Time sfx_linear / sfx_subm_conv per forced tile configuration on the heavy PTv3 shapes (config B).
python tools/gemm_cfg_bench.py [cfg ...]   (GPU only; -1 = cost model)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splatformer_amd import ptv3_ops as ops  # noqa: E402
from splatformer_amd.scenes import make_scene  # noqa: E402

LIN = [(37759, 1024, 256), (37759, 256, 1024), (37759, 768, 256), (37759, 256, 256), (14764, 2048, 512),
       (14764, 512, 2048), (70349, 512, 128), (70349, 128, 512)]


def timeit(fn, reps=10):
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
    cfgs = [int(c) for c in sys.argv[1:]] or [-1]
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    rows = []
    for M, N, K in LIN:
        x = torch.randn(M, K, device=dev, generator=g)
        w = torch.randn(N, K, device=dev, generator=g) / K ** 0.5
        b = torch.randn(N, device=dev, generator=g)
        out = torch.empty(M, N, device=dev)
        ref = None
        line = f"linear {M:6d}x{N:5d}x{K:5d}"
        for c in cfgs:
            ops.gemm_force_config(c, -1)
            us = timeit(lambda: ops.linear(x, w, b, out=out))
            if ref is None:
                ref = out.clone()
            err = float((out - ref).norm() / ref.norm())
            line += f"  cfg{c}: {us:8.1f} us {2 * M * N * K / us / 1e6:6.1f} TF{'' if err < 1e-5 else f' ERR {err:.1e}'}"
        rows.append(line)
        print(line, flush=True)
    sc = make_scene(100000, 1, seed=0)
    for n, C in [(37759, 256), (14764, 512), (70349, 128)]:
        grid = torch.floor(sc["means"][:n] * 384).int().to(dev)
        smap = ops.subm_neighbors(grid, None)
        x = torch.randn(grid.shape[0], C, device=dev, generator=g)
        w = torch.randn(C, 27 * C, device=dev, generator=g) * 0.02
        b = torch.randn(C, device=dev, generator=g)
        fl = 2.0 * (grid.shape[0] + smap.num_pairs) * C * C
        line = f"conv   {grid.shape[0]:6d}x{C:5d} P/N={smap.num_pairs / grid.shape[0]:.1f}"
        ref = None
        for c in cfgs:
            ops.gemm_force_config(c, -1)
            o = torch.empty(grid.shape[0], C, device=dev)
            us = timeit(lambda: ops.subm_conv(x, smap, w, b, out=o))
            if ref is None:
                ref = o.clone()
            err = float((o - ref).norm() / ref.norm())
            line += f"  cfg{c}: {us:8.1f} us {fl / us / 1e6:6.1f} TF{'' if err < 1e-5 else f' ERR {err:.1e}'}"
        print(line, flush=True)
    ops.gemm_force_config(-1, -1)


if __name__ == "__main__":
    main()
