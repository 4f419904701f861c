"""LDS-DMA GEMM on pre-split planes (sfx_gemm2) vs the register-staged GEMM (sfx_linear) on the config-B linear
shapes: per-launch time (HIP events, median of 20), fp32-equivalent TF/s (2 M N K / t), error vs fp64.
usage: python tools/gemm2_bench.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splatformer_amd import _lib  # noqa: E402
from splatformer_amd import ptv3_ops as ops  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gemm2_ops as g2  # noqa: E402

SHAPES = [(37759, 256, 768), (37759, 256, 1024), (37759, 1024, 256), (37759, 256, 256), (70349, 128, 512),
          (70349, 512, 128), (90434, 384, 96), (16000, 512, 2048), (14764, 512, 1536)]


def timeit(fn, reps=20, per_graph=10):
    """Median kernel time per call (us): `per_graph` calls captured in a HIP graph and replayed, so host launch
    overhead (tens of us per ctypes call) is not in the number."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(per_graph):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / per_graph)
    return statistics.median(ts)


def quick():
    """--quick: gemm2 kernel time only on the first four shapes (ablation variants via SFX_LIB)."""
    dev = torch.device("cuda:0")
    out = []
    for M, K, N in SHAPES[:4]:
        x = torch.randn(M, K, device=dev)
        w, b = torch.randn(N, K, device=dev), torch.randn(N, device=dev)
        xp = g2.split_planes(x)
        out.append(f"{M}x{K}x{N} {timeit(lambda: g2.linear2(xp, w, b)):7.1f}")
    print(os.path.basename(os.environ.get("SFX_LIB", "libsfx.so")) + ": " + " | ".join(out), flush=True)


def main():
    _lib.load()
    if "--quick" in sys.argv:
        return quick()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    for M, K, N in SHAPES:
        x = torch.randn(M, K, device=dev)
        lin = torch.nn.Linear(K, N).to(dev)
        w, b = lin.weight.detach(), lin.bias.detach()
        fl = 2.0 * M * N * K
        y_ref = (x.double() @ w.double().t() + b.double())
        t_old = timeit(lambda: ops.linear(x, w, b))
        xp = g2.split_planes(x)
        t_split = timeit(lambda: g2.split_planes(x))
        t_g2 = timeit(lambda: g2.linear2(xp, w, b))
        y_old, y_new = ops.linear(x, w, b), g2.linear2(xp, w, b)
        den = y_ref.norm()
        e_old = float((y_old.double() - y_ref).norm() / den)
        e_new = float((y_new.double() - y_ref).norm() / den)
        m_new = float((y_new.double() - y_ref).abs().max() / y_ref.abs().max())
        print(f"M={M:6d} K={K:4d} N={N:4d}: linear {t_old:7.1f} us ({fl / t_old / 1e6:6.1f} TF/s) | gemm2 {t_g2:7.1f} us "
              f"({fl / t_g2 / 1e6:6.1f} TF/s) + split {t_split:6.1f} us | speedup {t_old / t_g2:4.2f} "
              f"({t_old / (t_g2 + t_split):4.2f} incl split) | rel err old {e_old:.1e} new {e_new:.1e} "
              f"max {m_new:.1e}", flush=True)
        # gathered rows (centre tap of a SubM conv): every other row, a few -1
        idx = torch.arange(0, M, 2, device=dev, dtype=torch.int32)
        idx[::97] = -1
        yg = g2.linear2(xp, w, b, gather_idx=idx)
        xg = torch.where((idx >= 0)[:, None], x[idx.long().clamp(min=0)], torch.zeros((), device=dev))
        yg_ref = xg.double() @ w.double().t() + b.double()
        print(f"    gather: rel err {float((yg.double() - yg_ref).norm() / yg_ref.norm()):.1e}", flush=True)


if __name__ == "__main__":
    main()
