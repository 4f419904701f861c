"""Diagnostic: per-wave s_memtime totals of gemm2 (build with -DG2_STAMP=1 via tools/build_variant.sh, run with
SFX_LIB=<that .so>): total / stage waits+barriers / loop body / epilogues, in shader cycles, median and max over
waves.  usage: SFX_LIB=splatformer_amd/exp_stamp.so python tools/gemm2_stamps.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splatformer_amd import _lib  # noqa: E402
from splatformer_amd import ptv3_ops as ops  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gemm2_ops as g2  # noqa: E402

SHAPES = [(37759, 256, 768), (37759, 256, 1024), (37759, 1024, 256), (37759, 256, 256)]


def main():
    _lib.load()
    dev = torch.device("cuda:0")
    buf = torch.zeros(1024 * 8 * 4, dtype=torch.int64, device=dev)
    assert _lib.fn("sfx_gemm2_stamps")(_lib.C.c_void_p(buf.data_ptr())) == 0
    for M, K, N in SHAPES:
        x = torch.randn(M, K, device=dev)
        w, b = torch.randn(N, K, device=dev), torch.randn(N, device=dev)
        xp = g2.split_planes(x)
        for _ in range(5):
            buf.zero_()
            g2.linear2(xp, w, b)
        torch.cuda.synchronize()
        st = buf.view(-1, 4).cpu()
        st = st[st[:, 0] > 0].double()
        med, mx = st.median(0).values, st.max(0).values
        print(f"{M}x{K}x{N}: waves {st.shape[0]}  median total {med[0]:8.0f} wait {med[1]:8.0f} body {med[2]:8.0f} "
              f"epi {med[3]:8.0f} | max total {mx[0]:8.0f} wait {mx[1]:8.0f} body {mx[2]:8.0f} epi {mx[3]:8.0f}",
              flush=True)


if __name__ == "__main__":
    main()
