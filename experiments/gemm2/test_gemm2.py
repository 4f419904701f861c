"""LDS-DMA GEMM on pre-split fp16x2 planes (csrc/gemm2.hip: sfx_split_planes + sfx_gemm2) against fp64 torch:
the refiner's nn.Linear (reference pointtransformer_v3.py Block / MLP / SerializedAttention linears) at fp32
accuracy.  Ragged M / N / K (tails of the 256 x 128 x 32 tiles), gathered rows with empty (-1) entries, the
bias / BN-affine / GELU / residual epilogue."""
import pytest
import torch

import os
import sys

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ops():
    """The experiment's ops; needs SFX_LIB=experiments/gemm2/libsfx_gemm2.so (bash experiments/gemm2/build.sh)."""
    if "gemm2" not in os.environ.get("SFX_LIB", ""):
        pytest.skip("set SFX_LIB=experiments/gemm2/libsfx_gemm2.so")
    from splatformer_amd import _lib
    import gemm2_ops
    from splatformer_amd import ptv3_ops
    _lib.load()
    gemm2_ops.ACT_GELU = ptv3_ops.ACT_GELU
    return gemm2_ops


def _err(y, ref):
    return float((y.double() - ref).norm() / ref.norm())


@pytest.mark.parametrize("M,K,N", [(1, 128, 128), (300, 100, 200), (4097, 200, 132), (20000, 256, 768),
                                   (5000, 1024, 256), (777, 129, 64), (70001, 128, 512), (70001, 160, 256)])
def test_dense(ops, M, K, N):
    torch.manual_seed(M + K + N)
    dev = torch.device("cuda:0")
    x = torch.randn(M, K, device=dev) * torch.rand(M, 1, device=dev).mul(8).exp2()
    w = torch.randn(N, K, device=dev) / K ** 0.5
    b = torch.randn(N, device=dev)
    y = g2.linear2(x, w, b)
    ref = x.double() @ w.double().t() + b.double()
    assert _err(y, ref) < 2e-6  # fp32 arithmetic error (~1e-7 at these K)


def test_epilogue(ops):
    """bias + BN affine + GELU on the first 256 columns; then bias + residual (the two epilogue kinds)."""
    torch.manual_seed(1)
    dev = torch.device("cuda:0")
    for M in (3001, 70001):  # one tile per workgroup / persistent
        K, N = 160, 384
        x = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) / K ** 0.5
        b, sc, sh = torch.randn(N, device=dev), torch.rand(N, device=dev) + 0.5, torch.randn(N, device=dev)
        r = torch.randn(M, N, device=dev)
        y = g2.linear2(x, w, b, scale=sc, shift=sh, act=ops.ACT_GELU, act_ncols=256)
        z = (x.double() @ w.double().t() + b.double()) * sc.double() + sh.double()
        z[:, :256] = torch.nn.functional.gelu(z[:, :256])
        assert _err(y, z) < 2e-6
        y = g2.linear2(x, w, b, residual=r)
        ref = x.double() @ w.double().t() + b.double() + r.double()
        assert _err(y, ref) < 2e-6


def test_gather(ops):
    torch.manual_seed(2)
    dev = torch.device("cuda:0")
    M, K, N = 9000, 128, 256
    x = torch.randn(M, K, device=dev)
    w = torch.randn(N, K, device=dev) / K ** 0.5
    idx = torch.randint(0, M, (5003,), device=dev, dtype=torch.int32)
    idx[::13] = -1
    y = g2.linear2(x, w, None, gather_idx=idx)
    xg = torch.where((idx >= 0)[:, None], x[idx.long().clamp(min=0)], torch.zeros((), device=dev))
    ref = xg.double() @ w.double().t()
    assert _err(y, ref) < 2e-6
    assert torch.all(y[::13] == 0)
