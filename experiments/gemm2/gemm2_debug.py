"""Which gemm2 epilogue term is wrong: each term alone against fp64."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splatformer_amd import _lib  # noqa: E402
from splatformer_amd import ptv3_ops as ops  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gemm2_ops as g2  # noqa: E402


def main():
    _lib.load()
    dev = torch.device("cuda:0")
    torch.manual_seed(1)
    for M in (3001, 70001):
        K, N = 160, 384
        x = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) / K ** 0.5
        b, sc, sh = torch.randn(N, device=dev), torch.rand(N, device=dev) + 0.5, torch.randn(N, device=dev)
        r = torch.randn(M, N, device=dev)
        base = x.double() @ w.double().t()
        cases = {
            "plain": (dict(), base),
            "bias": (dict(bias=b), base + b.double()),
            "scale": (dict(scale=sc), base * sc.double()),
            "shift": (dict(shift=sh), base + sh.double()),
            "gelu": (dict(act=ops.ACT_GELU), torch.nn.functional.gelu(base)),
            "gelu256": (dict(act=ops.ACT_GELU, act_ncols=256),
                        torch.cat([torch.nn.functional.gelu(base[:, :256]), base[:, 256:]], 1)),
            "res": (dict(residual=r), base + r.double()),
        }
        for name, (kw, ref) in cases.items():
            kw = dict(kw)
            bias = kw.pop("bias", None)
            y = g2.linear2(x, w, bias, **kw)
            e = (y.double() - ref).abs()
            bad = (e > 1e-4 * ref.abs().max()).nonzero()
            print(f"M={M} {name:8s} rel {float(e.norm() / ref.norm()):.2e} bad {bad.shape[0]} first {bad[:4].tolist()}",
                  flush=True)


if __name__ == "__main__":
    main()
