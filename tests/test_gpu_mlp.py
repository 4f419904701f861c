"""Fused Block MLP tail (csrc/mlp.hip, sfx_block_mlp): Y = X + fc2(GELU(fc1(LN2(X)))) -- reference Block.forward
restated in calflops.py:72-82 (norm2 -> mlp -> + shortcut) -- against the fp64 torch reference of the same ops,
at the bar of the GEMM family's tests (relative L2 <= 2e-6, each row's error within 4x that of torch's fp32 CPU
evaluation of the unfused ops), for every channel count the kernel serves and ragged point counts."""
import copy

import pytest
import torch
import torch.nn.functional as F

from splatformer_amd import ptv3_ops as ops
from test_gpu_ptv3 import rel_l2

pytestmark = pytest.mark.gpu


def _mods(C, seed):
    g = torch.Generator().manual_seed(seed)
    ln = torch.nn.LayerNorm(C)
    fc1, fc2 = torch.nn.Linear(C, 4 * C), torch.nn.Linear(4 * C, C)
    with torch.no_grad():
        ln.weight.copy_(torch.rand(C, generator=g) + 0.5)
        ln.bias.copy_(torch.randn(C, generator=g) * 0.1)
        for lin in (fc1, fc2):
            lin.weight.copy_(torch.randn(lin.weight.shape, generator=g) / lin.weight.shape[1] ** 0.5)
            lin.bias.copy_(torch.randn(lin.bias.shape, generator=g) * 0.1)
    return ln, fc1, fc2


@torch.no_grad()
def _ref(x, ln, fc1, fc2, dtype):
    x = x.to(dtype)
    h = F.layer_norm(x, (x.shape[1],), ln.weight.to(dtype), ln.bias.to(dtype), ln.eps)
    m = F.gelu(F.linear(h, fc1.weight.to(dtype), fc1.bias.to(dtype)))
    return x + F.linear(m, fc2.weight.to(dtype), fc2.bias.to(dtype))


@pytest.mark.parametrize("C", ops.MLP_CHANNELS)
@pytest.mark.parametrize("M", [1, 63, 4097])
def test_block_mlp_matches_fp64(device, C, M):
    _check_fp64(device, C, M)


# (C, M) whose last round of workgroups is at most half full on 256 CUs: C = 256 one 64-point workgroup per CU,
# C = 128 two 64-point (both split their tail), C <= 96 two 128-point ones (not split: the unsplit path again)
SPLIT_CASES = [(256, 256 * 64 + 1000), (256, 256 * 64 + 5000), (256, 2 * 256 * 64 + 777), (128, 512 * 64 + 2000),
               (96, 512 * 128 + 3000), (96, 512 * 128 + 20000), (64, 512 * 128 + 5000)]


@pytest.mark.parametrize("C,M", SPLIT_CASES)
def test_block_mlp_split_tail(device, C, M):
    """Launches whose last round is at most half full: the tail runs as 4- / 3- / 2-way hidden-chunk splits + the
    fixed-order combine (csrc/mlp.hip run_eval_split) -- the bar of the unsplit kernel -- and the combine's row
    exponents equal sfx_subm_rowexp of the output."""
    _check_fp64(device, C, M)
    ln, fc1, fc2 = _mods(C, 7 * C)
    x = torch.randn(M, C, generator=torch.Generator().manual_seed(M)) * 2.0
    mods = [m.to(device) for m in (ln, fc1, fc2)]
    e = torch.full((M,), -999, device=device, dtype=torch.int32)
    y = ops.block_mlp(x.to(device), *mods, rowexp=e)
    assert torch.equal(e.cpu(), ops.subm_rowexp(y).cpu())


def _check_fp64(device, C, M):
    ln, fc1, fc2 = _mods(C, C + M)
    g = torch.Generator().manual_seed(M)
    x = torch.randn(M, C, generator=g) * 2.0
    x[::3] *= 1e3   # rows of very different magnitudes (LayerNorm normalises them; the residual keeps them)
    x[1::5] *= 1e-3
    ref = _ref(x, ln, fc1, fc2, torch.float64)
    r32 = _ref(x, ln, fc1, fc2, torch.float32).double()
    lnd, f1d, f2d = ln.to(device), fc1.to(device), fc2.to(device)
    y = ops.block_mlp(x.to(device), lnd, f1d, f2d).cpu().double()
    assert torch.isfinite(y).all()
    # the MLP branch (Y - X) is what the kernel computes; the residual add is exact up to one rounding
    br, bh, b32 = ref - x.double(), y - x.double(), r32 - x.double()
    # (rows scaled by 1e3 carry the fp32 rounding of the residual add: the bar is relative to torch's fp32 error)
    assert rel_l2(bh, br) <= max(2e-6, 2 * rel_l2(b32, br)), (rel_l2(bh, br), rel_l2(b32, br))
    e_row = (bh - br).norm(dim=1) / br.norm(dim=1).clamp_min(1e-30)
    e32 = (b32 - br).norm(dim=1) / br.norm(dim=1).clamp_min(1e-30)
    assert bool((e_row <= 4 * e32 + 1e-6).all()), float((e_row - 4 * e32).max())


def test_block_mlp_strided_output_and_cache(device):
    """Writes into a column slice of a wider buffer (the last Block writes into the head input, ld 120), and the
    packed weights are rebuilt when a weight changes in place."""
    C, M = 96, 1000
    ln, fc1, fc2 = [m.to(device) for m in _mods(C, 3)]
    x = torch.randn(M, C, generator=torch.Generator().manual_seed(1)).to(device)
    buf = torch.full((M, 120), 7.0, device=device)
    ops.block_mlp(x, ln, fc1, fc2, out=buf[:, :C])
    cpu = lambda m: copy.deepcopy(m).cpu()  # (Module.cpu() moves in place)
    ref = _ref(x.cpu(), cpu(ln), cpu(fc1), cpu(fc2), torch.float64)
    assert rel_l2(buf[:, :C].cpu().double() - x.cpu().double(), ref - x.cpu().double()) < 2e-6
    assert bool((buf[:, C:] == 7.0).all())
    with torch.no_grad():
        fc1.weight.mul_(0.5)  # in-place change: bumps the version, so the packed stream is rebuilt
    y2 = ops.block_mlp(x, ln, fc1, fc2)
    ref2 = _ref(x.cpu(), cpu(ln), cpu(fc1), cpu(fc2), torch.float64)
    assert rel_l2(y2.cpu().double() - x.cpu().double(), ref2 - x.cpu().double()) < 2e-6


def test_block_fused_equals_unfused(device):
    """Block.run with the fused tail vs the LayerNorm + two-GEMM form (SFX_MLP_FUSED=0 path)."""
    C, M = 128, 3001
    ln, fc1, fc2 = [m.to(device) for m in _mods(C, 5)]
    x = torch.randn(M, C, generator=torch.Generator().manual_seed(2)).to(device)
    y = ops.block_mlp(x, ln, fc1, fc2)
    h = ops.layernorm(x, ln.weight, ln.bias, ln.eps)
    m = ops.linear(h, fc1.weight, fc1.bias, act=ops.ACT_GELU)
    y0 = ops.linear(m, fc2.weight, fc2.bias, residual=x)
    assert rel_l2((y - x).cpu(), (y0 - x).cpu()) < 4e-6


@pytest.mark.parametrize("C", ops.MLP_CHANNELS)
@pytest.mark.parametrize("waves,hs", [("4", "0"), ("4", "1"), ("4", "2"), ("8", "0"), ("8", "1")])
def test_block_mlp_launch_variants(device, monkeypatch, C, waves, hs):
    """Every workgroup shape sfx_block_mlp can launch (SFX_MLP_WAVES: 128- / 256-point workgroups at C <= 128;
    SFX_MLP_HS: the hidden split -- a wave pair per 32 points, partial fc2 sums added through LDS -- at no C, the
    default C = 128 / 256, every C) at the fp64 bar of test_block_mlp_matches_fp64, on a ragged point count."""
    monkeypatch.setenv("SFX_MLP_WAVES", waves)
    monkeypatch.setenv("SFX_MLP_HS", hs)
    M = 3001
    ln, fc1, fc2 = _mods(C, 7 * C)
    x = torch.randn(M, C, generator=torch.Generator().manual_seed(C)) * 2.0
    x[::3] *= 1e3
    ref = _ref(x, ln, fc1, fc2, torch.float64)
    r32 = _ref(x, ln, fc1, fc2, torch.float32).double()
    y = ops.block_mlp(x.to(device), ln.to(device), fc1.to(device), fc2.to(device)).cpu().double()
    br, bh, b32 = ref - x.double(), y - x.double(), r32 - x.double()
    assert torch.isfinite(y).all()
    assert rel_l2(bh, br) <= max(2e-6, 2 * rel_l2(b32, br)), (rel_l2(bh, br), rel_l2(b32, br))
    e_row = (bh - br).norm(dim=1) / br.norm(dim=1).clamp_min(1e-30)
    e32 = (b32 - br).norm(dim=1) / br.norm(dim=1).clamp_min(1e-30)
    assert bool((e_row <= 4 * e32 + 1e-6).all()), float((e_row - 4 * e32).max())


@pytest.mark.parametrize("C", ops.MLP_CHANNELS)
def test_block_mlp_rowexp(device, C):
    """The MLP epilogue's row exponents of its output (for the next fused SubM conv) equal sfx_subm_rowexp of the
    output, bit for bit, incl. zero rows (127)."""
    M = 3001
    ln, fc1, fc2 = _mods(C, 7 * C)
    g = torch.Generator().manual_seed(C)
    x = torch.randn(M, C, generator=g) * 2.0
    x[::7] *= 1e4
    x[3::11] *= 1e-4
    mods = [m.to(device) for m in (ln, fc1, fc2)]
    e = torch.full((M,), -999, device=device, dtype=torch.int32)
    y = ops.block_mlp(x.to(device), *mods, rowexp=e)
    assert torch.equal(e.cpu(), ops.subm_rowexp(y).cpu())
    # zero output rows (x = 0 and a zero fc2): exponent 127
    with torch.no_grad():
        mods[2].weight.zero_()
        mods[2].bias.zero_()
    xz = torch.zeros(64, C, device=device)
    ez = torch.empty(64, device=device, dtype=torch.int32)
    yz = ops.block_mlp(xz, *mods, rowexp=ez)
    assert float(yz.abs().max()) == 0.0 and bool((ez == 127).all())
