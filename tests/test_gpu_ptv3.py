"""HIP PTv3 refiner (libsfx) vs the CPU oracle (oracle/ptv3_ref.py, oracle/serialize_ref.py).

Integer/index work (serialization codes/order/inverse, neighbour maps, pooling
clusters) is compared bit-exactly; fp32 features within the north-star
tolerance: relative L2 error <= 1e-5 on the backbone feature and the refined
Gaussians, per-op 1e-5 relative.
"""
import numpy as np
import pytest
import torch

from oracle import ptv3_ref, serialize_ref
from splatformer_amd import ptv3_ops as ops
from splatformer_amd.feature_predictor import FeaturePredictor
from splatformer_amd.scenes import make_scene, to_device

pytestmark = pytest.mark.gpu


def rel_l2(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


# ---- ops --------------------------------------------------------------------------
@pytest.mark.parametrize("M,N,K,act", [(1000, 64, 23, 1), (3000, 96, 64, 0), (517, 384, 128, 2), (257, 512, 2048, 0),
                                       (100, 23, 768, 3)])
def test_linear_vs_torch(device, M, N, K, act):
    g = torch.Generator().manual_seed(M + N)
    x = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    sc = torch.rand(N, generator=g) + 0.5
    sh = torch.randn(N, generator=g)
    res = torch.randn(M, N, generator=g)
    ref = (x @ w.T + b) * sc + sh
    ref = [ref, torch.nn.functional.gelu(ref), torch.relu(ref), torch.tanh(ref)][act] + res
    y = ops.linear(x.to(device), w.to(device), b.to(device), act=act, scale=sc.to(device), shift=sh.to(device),
                   residual=res.to(device))
    assert rel_l2(y.cpu(), ref) < 2e-6


def _slot_value(device, slot):
    """max over the sub-slots of an amax slot (ops.new_amax ring) carrying its tag."""
    buf = ops._amax_state[device][0] if device in ops._amax_state else ops._amax_state[torch.device(device)][0]
    off = (slot[0] - buf.data_ptr()) // 8
    w = buf[off:off + ops.AMAX_SUB].cpu()
    vals = [int(v) & 0xFFFFFFFF for v in w.tolist() if (int(v) >> 32) & 0xFFFFFFFF == slot[1]]
    return max(torch.tensor(vals, dtype=torch.int64).to(torch.int32).view(torch.float32).tolist()) if vals else 0.0


@pytest.mark.parametrize("M,N,K", [(4097, 96, 96), (1, 128, 128), (31, 100, 64), (3001, 288, 96), (2500, 384, 128),
                                   (777, 64, 128)])
def test_linear_narrow_cases(device, M, N, K):
    """The refine's narrow dense linears (K in {64, 96, 128}): bias, GELU on the first columns only, residual
    (also in place), max |Y| published to a slot, strided input / output, ragged M and N, rows of very different
    magnitudes -- each row within 2x (+1e-7) of torch's fp32 CPU error against fp64."""
    g = torch.Generator().manual_seed(M * 7 + N + K)
    xb = torch.randn(M, K + 8, generator=g)
    xb[::3] *= 1e4
    xb[1::7] *= 1e-5
    x = xb[:, 4:4 + K]
    w = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    res = torch.randn(M, N, generator=g)
    ac = N // 2
    z = x.double() @ w.double().T + b.double()
    ref = torch.cat([torch.nn.functional.gelu(z[:, :ac]), z[:, ac:]], 1) + res.double()
    z32 = x @ w.T + b
    f32 = (torch.cat([torch.nn.functional.gelu(z32[:, :ac]), z32[:, ac:]], 1) + res).double()
    xd = xb.to(device)[:, 4:4 + K]
    out = torch.full((M, N + 12), 7.0, device=device)
    y, slot = ops.linear(xd, w.to(device), b.to(device), act=ops.ACT_GELU, act_ncols=ac, residual=res.to(device),
                         out=out[:, :N], y_amax=True)
    yh = y.cpu().double()
    rn = ref.norm(dim=1).clamp_min(1e-30)
    e_hip, e_f32 = (yh - ref).norm(dim=1) / rn, (f32 - ref).norm(dim=1) / rn
    assert bool((e_hip <= 2 * e_f32 + 1e-7).all()), float((e_hip - 2 * e_f32).max())
    assert bool((out[:, N:] == 7.0).all())
    amax = _slot_value(device, slot)
    assert abs(amax - float(yh.abs().max())) <= 1e-6 * float(yh.abs().max())
    # in-place residual (Y = R): x W^T + b added onto the residual rows
    r2 = res.to(device).clone()
    ops.linear(xd, w.to(device), b.to(device), residual=r2, out=r2)
    ref2 = z + res.double()
    assert rel_l2(r2.cpu(), ref2) <= 2 * rel_l2((x @ w.T + b + res), ref2) + 1e-7


def test_gelu_fitted_tail_accuracy(device):
    """The GEMM epilogue's GELU (gemm_common.h gelu_erf: Phi from one fitted tail exponent, shared by the fused
    MLP) against fp64 erf-GELU over [-12, 12], at 0 / +-tiny, and far in the tails (one row of |x| up to 1e4: the
    negative tail is exactly 0 below -5.65): |dGELU| <= 4e-7 max(1, |x|) -- the fit's 6e-8 on Phi plus the
    fp16x2 split of the identity product's input (x = h + l to 2^-22 = 2.4e-7 relative)."""
    x = torch.linspace(-12.0, 12.0, 4096 * 64, dtype=torch.float64)
    x[:8] = torch.tensor([0.0, 1e-30, -1e-30, 1e-8, -1e-8, 5.65, -5.65, 0.5])
    x[64:128] = torch.cat([-torch.logspace(0.8, 4, 32, dtype=torch.float64), torch.logspace(0.8, 4, 32, dtype=torch.float64)])
    x32 = x.float().reshape(4096, 64)
    eye = torch.eye(64)
    y = ops.linear(x32.to(device), eye.to(device), None, act=ops.ACT_GELU).cpu().double().flatten()
    xd = x32.double().flatten()
    ref = 0.5 * xd * (1.0 + torch.erf(xd / 2 ** 0.5))
    err = (y - ref).abs() / xd.abs().clamp_min(1.0)
    assert float(err.max()) <= 4e-7, (float(err.max()), float(xd[int(err.argmax())]))
    assert float(y[0]) == 0.0 and torch.isfinite(y).all()
    assert bool((y[64:96] == 0.0).all()), y[64:96]  # x <= -6.3: GELU underflows to exactly 0, as fp32 erf does


@pytest.mark.parametrize("scale", [1.0, 1e-30, 1e30])
def test_linear_split_precision_is_fp32(device, scale):
    """The fp16x2 split GEMM (default for K >= 64: a power-of-two scale per operand row -- A' rows chosen online
    by the kernel, W rows by the cached pre-split --, two fp16 terms per operand, three term products) is as
    accurate as fp32 arithmetic: its error against an fp64 product is at most that of torch's fp32 CPU GEMM
    (x1.5), at operand magnitudes 1e+-30 (the scales absorb them)."""
    g = torch.Generator().manual_seed(7)
    M, N, K = 2000, 384, 1024
    x = torch.randn(M, K, generator=g) * scale
    w = torch.randn(N, K, generator=g) / K ** 0.5
    ref = x.double() @ w.double().T
    y = ops.linear(x.to(device), w.to(device), None).cpu()
    e_hip = rel_l2(y, ref)
    e_f32 = rel_l2(x @ w.T, ref)
    assert torch.isfinite(y).all()
    assert e_hip <= 1.5 * e_f32, (e_hip, e_f32)


@pytest.mark.parametrize("M,N,K", [(3000, 384, 128), (2000, 1024, 256), (777, 96, 96)])
def test_linear_reference_precision_mode(device, M, N, K):
    """ops.precision("amp") (include/sfx.h sfx_set_precision(1): the class of the reference's fp16 autocast
    training, train.py:240) forms one fp16 product per block -- operands rounded to fp16 (round-to-nearest; the
    kernel's power-of-two row scales change no rounding of a normal value), exact products, fp32 accumulation:
    within 2x (+1e-7) of torch's fp32 error on the fp16-rounded operands, as far from the exact product as fp16
    operand rounding puts it, and the mode is restored on exit."""
    g = torch.Generator().manual_seed(M + K)
    x = torch.randn(M, K, generator=g) * 3
    w = torch.randn(N, K, generator=g) / K ** 0.5
    x16, w16 = x.half().float(), w.half().float()
    ref16 = x16.double() @ w16.double().T
    with ops.precision("amp"):
        assert ops.get_precision() == "amp"
        y = ops.linear(x.to(device), w.to(device), None).cpu()
    assert ops.get_precision() == "fp32"
    assert rel_l2(y, ref16) <= 2 * rel_l2(x16 @ w16.T, ref16) + 1e-7
    e = rel_l2(y, x.double() @ w.double().T)
    assert 5e-5 < e < 1e-3, e
    y32 = ops.linear(x.to(device), w.to(device), None).cpu()  # default mode again: fp32-accurate
    assert rel_l2(y32, x.double() @ w.double().T) <= 1.5 * rel_l2(x @ w.T, x.double() @ w.double().T) + 1e-7


@pytest.mark.parametrize("span", [10, 20])
def test_linear_split_rows_wide_dynamic_range(device, span):
    """Rows whose magnitudes span 2^-span .. 2^span (of each other) keep fp32 accuracy row by row: every row's
    error against fp64 is within 2x (+ fp32 rounding of the row's own scale) of torch's fp32 CPU GEMM's."""
    g = torch.Generator().manual_seed(span)
    M, N, K = 1024, 256, 512
    e = torch.linspace(-span, span, M)
    x = torch.randn(M, K, generator=g) * torch.exp2(e)[:, None]
    w = torch.randn(N, K, generator=g) / K ** 0.5
    ref = x.double() @ w.double().T
    y = ops.linear(x.to(device), w.to(device), None).cpu().double()
    f32 = (x @ w.T).double()
    rn = ref.norm(dim=1)
    e_hip = (y - ref).norm(dim=1) / rn
    e_f32 = (f32 - ref).norm(dim=1) / rn
    worst = int(torch.argmax(e_hip / (e_f32 + 1e-7)))
    assert bool((e_hip <= 2 * e_f32 + 1e-7).all()), \
        f"row {worst} (2^{float(e[worst]):.1f}): rel err {float(e_hip[worst]):.3e} vs fp32 {float(e_f32[worst]):.3e}"


def test_linear_gather_is_subm_conv(device):
    n, C = 4000, 64
    s = make_scene(n, 1, seed=3, unique_voxels=True)
    grid = torch.floor(s["means"] * 384).int()
    batch = torch.zeros(grid.shape[0], dtype=torch.int64)
    nbr_ref = ptv3_ref.subm_neighbors(grid, batch)
    smap = ops.subm_neighbors(grid.to(device), None)
    nbr = smap.nbr
    assert torch.equal(nbr.cpu().long(), nbr_ref)
    # offset-major pair lists: exactly the non-centre (out, in) pairs, output rows ascending per offset
    off = smap.pair_off
    pin, pout = smap.pair_in.cpu().long(), smap.pair_out.cpu().long()
    for k in range(27):
        rows = torch.nonzero(nbr_ref[:, k] >= 0).flatten() if k != 13 else torch.zeros(0, dtype=torch.long)
        assert torch.equal(pout[off[k]:off[k + 1]], rows)
        assert torch.equal(pin[off[k]:off[k + 1]], nbr_ref[rows, k])
    assert off[27] == int((nbr_ref >= 0).sum()) - grid.shape[0]
    g = torch.Generator().manual_seed(0)
    x = torch.randn(grid.shape[0], C, generator=g)
    w = torch.randn(C, 3, 3, 3, C, generator=g) * 0.05
    b = torch.randn(C, generator=g)
    ref = ptv3_ref.subm_conv(x, nbr_ref, w, b)
    y = ops.linear(x.to(device), w.to(device).reshape(C, 27 * C), b.to(device), gather_idx=nbr)
    assert rel_l2(y.cpu(), ref) < 2e-6
    for cin in (64, 96, 256):  # offset-major sparse conv (centre GEMM + atomic pair GEMM)
        xx = torch.randn(grid.shape[0], cin, generator=g)
        ww = torch.randn(cin, 3, 3, 3, cin, generator=g) * 0.05
        bb = torch.randn(cin, generator=g)
        ref2 = ptv3_ref.subm_conv(xx, nbr_ref, ww, bb)
        y2 = ops.subm_conv(xx.to(device), smap, ww.to(device), bb.to(device))
        assert rel_l2(y2.cpu(), ref2) < 2e-6


@pytest.mark.parametrize("C", [64, 96, 128, 256, 512, 30])
def test_segment_max_affine_act(device, C):
    """Pooling's segment max -> BN affine -> GELU (sfx_segment_max_affine_act; one wave per cluster for C % 4 == 0,
    the per-cluster workgroup form for C = 30) against torch: runs of 1-8 rows in a permuted order, ragged m."""
    g = torch.Generator().manual_seed(C)
    m = 5003
    lens = torch.randint(1, 9, (m,), generator=g)
    idx_ptr = torch.zeros(m + 1, dtype=torch.int64)
    idx_ptr[1:] = torch.cumsum(lens, 0)
    n = int(idx_ptr[-1])
    sidx = torch.randperm(n, generator=g)
    x = torch.randn(n, C, generator=g)
    sc, sh = torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g)
    y = ops.segment_max_affine_act(x.to(device), idx_ptr.int().to(device), sidx.int().to(device), m, sc.to(device),
                                   sh.to(device), ops.ACT_GELU)
    seg = torch.repeat_interleave(torch.arange(m), lens)
    mx = torch.full((m, C), -float("inf")).scatter_reduce(0, seg[:, None].expand(n, C), x[sidx], "amax")
    ref = torch.nn.functional.gelu(mx * sc + sh)
    assert rel_l2(y.cpu(), ref) < 1e-6


@pytest.mark.parametrize("n", [1, 255, 256, 257, 6000, 70000])
@pytest.mark.parametrize("centre", [False, True])
def test_subm_pair_lists_match_flag_scan(device, n, centre):
    """sfx_subm_pair_lists (ABI v16: per-workgroup counts + one scan of 27 ceil(n/256) counts, pair_pos written with
    the lists) equals sfx_subm_pairs + sfx_subm_pair_pos (flags over [27][n], one scan, fill) bit for bit -- lists,
    per-offset prefixes and the inverted index -- on ragged n (one point, workgroup edges) with duplicate voxels."""
    from splatformer_amd import _lib
    from splatformer_amd.ptv3_ops import call, ptr, stream
    s = make_scene(n, 1, seed=7, unique_voxels=False)
    grid = torch.floor(s["means"] * 256).int().to(device)
    nbr = ops.subm_neighbors(grid, None, with_pairs=False).nbr
    cap = max(1, 27 * n)
    res = []
    for new in (False, True):
        pin = torch.full((cap,), -7, device=device, dtype=torch.int32)
        pout = torch.full((cap,), -7, device=device, dtype=torch.int32)
        off = torch.empty(28, device=device, dtype=torch.int32)
        pos = torch.empty(n, 27, device=device, dtype=torch.int32)
        if new:
            ws = _lib.workspace(_lib.fn("sfx_subm_pair_lists_workspace_bytes")(n), device)
            cpos = torch.empty(n, 32, device=device, dtype=torch.int32)
            call("sfx_subm_pair_lists", n, ptr(nbr), ptr(ws), ws.numel(), ptr(pin), ptr(pout), ptr(off), ptr(pos),
                 ptr(cpos), 1 if centre else 0, stream())
        else:
            ws = _lib.workspace(_lib.fn("sfx_subm_pairs_workspace_bytes")(n), device)
            call("sfx_subm_pairs", n, ptr(nbr), ptr(ws), ws.numel(), ptr(pin), ptr(pout), ptr(off),
                 1 if centre else 0, stream())
            call("sfx_subm_pair_pos", n, int(off[27].item()), ptr(pout), ptr(off), ptr(pos), stream())
        torch.cuda.synchronize()
        res.append((pin.cpu(), pout.cpu(), off.cpu(), pos.cpu()))
    for a, b in zip(*res):
        assert torch.equal(a, b)
    # the compacted positions: each row's present pair indices in ascending offset order, -1 after, count in column 31
    cp, pos = cpos.cpu(), res[1][3]
    cnt = (pos >= 0).sum(1)
    assert torch.equal(cp[:, 31], cnt.int())
    for i in range(0, n, max(1, n // 97)):
        want = pos[i][pos[i] >= 0]
        c = int(cnt[i])
        assert torch.equal(cp[i, :c], want) and bool((cp[i, c:31] == -1).all())
    off = res[1][2]
    assert int(off[27]) == int(((nbr >= 0).sum() - (0 if centre else (nbr[:, 13] >= 0).sum())).item())


@pytest.mark.parametrize("centre,unique", [(False, True), (True, True), (True, False)])
def test_subm_conv_partials_atomic_free(device, centre, unique):
    """Atomic-free SubM conv (sfx_subm_conv_partials + sfx_subm_pair_pos + sfx_cpe_residual_ln_pairs): the inverted
    pair index names every pair, the per-row sum in ascending offset order equals the oracle conv, the fused
    cpe/residual/LN tail equals the unfused one on that sum bit for bit, and two runs agree bit for bit.
    centre=True: the eval forward's lists with the centre offset (one pair launch, bias-only T; ABI v15), incl.
    duplicate voxels (the centre pair's input is the voxel's lowest-index point)."""
    n = 6000
    s = make_scene(n, 1, seed=5, unique_voxels=unique)
    grid = torch.floor(s["means"] * 320).int()
    nbr_ref = ptv3_ref.subm_neighbors(grid, torch.zeros(grid.shape[0], dtype=torch.int64))
    smap = ops.subm_neighbors(grid.to(device), None, centre=centre)
    pl = smap.lists(centre)
    off = pl.pair_off
    pos = pl.pair_pos.cpu().long()
    pout = pl.pair_out.cpu().long()
    assert int((pos >= 0).sum()) == off[27] and bool((pos[:, 13] >= 0).all() if centre else (pos[:, 13] < 0).all())
    for k in range(27):
        if k == 13 and not centre:
            continue
        p = torch.arange(off[k], off[k + 1])
        assert torch.equal(pos[pout[p], k], p)
        assert torch.equal(pos[:, k] >= 0, nbr_ref[:, k] >= 0)
    g = torch.Generator().manual_seed(4)
    for C in (64, 96, 128, 256):
        x = torch.randn(grid.shape[0], C, generator=g)
        w = torch.randn(C, 3, 3, 3, C, generator=g) * 0.05
        b = torch.randn(C, generator=g)
        ga, be = torch.randn(C, generator=g), torch.randn(C, generator=g)
        g1, b1 = torch.randn(C, generator=g), torch.randn(C, generator=g)
        xd, wd, bd = x.to(device), w.to(device), b.to(device)
        sp = ops.subm_conv(xd, smap, wd, bd, partials=True)
        t = sp.total()
        assert rel_l2(t.cpu(), ptv3_ref.subm_conv(x, nbr_ref, w, b)) < 2e-6
        args = (ga.to(device), be.to(device), g1.to(device), b1.to(device), 1e-5)
        xo, h = ops.cpe_residual_ln(sp, xd, *args)
        xo_u, h_u = ops.cpe_residual_ln(t, xd, *args)
        assert torch.equal(xo, xo_u) and torch.equal(h, h_u)
        if sp.cpos is not None:  # the compacted-position LayerNorm equals the [n][27] one bit for bit
            sp_k = ops.SubmPartials(sp.centre, sp.partials, sp.pair_pos, sp.num_pairs, ldt=sp.ldt)
            xo_k, h_k = ops.cpe_residual_ln(sp_k, xd, *args)
            assert torch.equal(xo, xo_k) and torch.equal(h, h_k)
        sp2 = ops.subm_conv(xd, smap, wd, bd, partials=True)
        xo2, h2 = ops.cpe_residual_ln(sp2, xd, *args)
        assert torch.equal(xo, xo2) and torch.equal(h, h2)


@pytest.mark.parametrize("C", [64, 96, 128])
@pytest.mark.parametrize("n,centre", [(6000, True), (4133, False), (1, True), (129, True)])
def test_cpe_ln_qkv_fused(device, C, n, centre):
    """sfx_cpe_ln_qkv_pairs (pair sums + LN_cpe + shortcut + norm1 + qkv in one launch, norm1's output on chip) vs
    the unfused HIP path (sfx_cpe_residual_ln_pairs + the qkv GEMM): x1 bit for bit (same LayerNorm arithmetic), qkv
    against the fp64 product of the unfused path's h (fp16x2 terms: fp32-level error), the published amax bounding
    |qkv|; ragged tile (n % 128 != 0), a single point, both pair-list kinds."""
    s = make_scene(n, 1, seed=9, unique_voxels=False)
    grid = torch.floor(s["means"] * 320).int()
    smap = ops.subm_neighbors(grid.to(device), None, centre=centre)
    g = torch.Generator().manual_seed(C + n)
    x = torch.randn(n, C, generator=g).to(device)
    w = (torch.randn(C, 3, 3, 3, C, generator=g) * 0.05).to(device)
    b = torch.randn(C, generator=g).to(device)
    ln = [torch.randn(C, generator=g).to(device) for _ in range(4)]
    lin = torch.nn.Linear(C, 3 * C).to(device)
    with torch.no_grad():
        lin.weight.copy_(torch.randn(3 * C, C, generator=g) * C ** -0.5)
        lin.bias.copy_(torch.randn(3 * C, generator=g) * 0.1)
    sp = ops.subm_conv(x, smap, w, b, partials=True)
    x1_u, h_u = ops.cpe_residual_ln(sp, x, *ln, 1e-5)
    x1, qkv, slot = ops.cpe_ln_qkv(sp, x, *ln, 1e-5, lin)
    assert torch.equal(x1, x1_u)
    ref = h_u.double() @ lin.weight.double().T + lin.bias.double()
    e = rel_l2(qkv.double(), ref)
    e_gemm = rel_l2(ops.linear(h_u, lin.weight, lin.bias).double(), ref)
    print(f"\n[cpe_ln_qkv C={C} n={n}] qkv rel L2 vs fp64: fused {e:.2e}, qkv GEMM {e_gemm:.2e}")
    assert e < 2e-6
    assert _slot_value(device, slot) >= float(qkv.abs().max())


@pytest.mark.parametrize("C", [64, 96, 128, 256])
@pytest.mark.parametrize("n,unique,sep", [(6000, True, False), (4133, False, True), (1, True, False),
                                          (20011, False, False)])
def test_subm_cpe_ln_fused(device, C, n, unique, sep):
    """sfx_subm_cpe_ln (the eval CPE: conv summed over all 27 offsets in MFMA registers + LN_cpe + shortcut + norm1
    in one launch, the default path) against the fp64 oracle (ptv3_ref.subm_conv then the two LayerNorms) --
    relative L2 <= 2e-6 on x1 and h -- and against the pair-GEMM path; duplicate voxels, row counts not a multiple
    of the workgroup's points, a separate conv input (the first decoder Block's stale skip feature), a single
    point; rows of very different magnitude (one fp16x2 scale per output point over its neighbours' rows); two runs
    bitwise equal."""
    s = make_scene(max(n, 64), 1, seed=n + C, unique_voxels=unique)
    grid = torch.floor(s["means"][:n] * 256).int()
    n = grid.shape[0]
    nbr_ref = ptv3_ref.subm_neighbors(grid, torch.zeros(n, dtype=torch.int64))
    smap = ops.subm_neighbors(grid.to(device), None, with_pairs=False)
    g = torch.Generator().manual_seed(C)
    x = torch.randn(n, C, generator=g) * torch.exp2(torch.randint(-8, 9, (n, 1), generator=g).float())
    xc = torch.randn(n, C, generator=g) if sep else x
    wf = torch.randn(C, 27 * C, generator=g) * 0.05
    bf = torch.randn(C, generator=g)
    ga, be = torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g)
    g1, b1 = torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g)
    dev = lambda t: t.to(device).contiguous()
    wpk, winv = ops.subm_cpe_pack(dev(wf))
    args = (dev(bf), dev(ga), dev(be), dev(g1), dev(b1), 1e-5)
    x1, h = ops.subm_cpe_ln(dev(xc), dev(x), smap, wpk, winv, *args)
    x1b, hb = ops.subm_cpe_ln(dev(xc), dev(x), smap, wpk, winv, *args)
    assert torch.equal(x1, x1b) and torch.equal(h, hb)
    # fp64 reference: W' as [C, 27, C] = spconv [Cout, 3, 3, 3, Cin]
    w5 = wf.double().view(C, 3, 3, 3, C)
    t = ptv3_ref.subm_conv(xc.double(), nbr_ref, w5, bf.double())
    ln = lambda v, gg, bb: torch.nn.functional.layer_norm(v, (C,), gg.double(), bb.double(), 1e-5)
    x1r = x.double() + ln(t, ga, be)
    hr = ln(x1r, g1, b1)
    e1, e2 = rel_l2(x1.cpu().double(), x1r), rel_l2(h.cpu().double(), hr)
    assert e1 < 2e-6 and e2 < 2e-6, (e1, e2)
    # the pair-GEMM path on the same inputs
    sp = ops.subm_conv(dev(xc), smap, dev(wf.view(C, 3, 3, 3, C)), dev(bf), partials=True)
    xo, ho = ops.cpe_residual_ln(sp, dev(x), *args[1:])
    assert rel_l2(x1.cpu(), xo.cpu()) < 2e-6 and rel_l2(h.cpu(), ho.cpu()) < 2e-6


@pytest.mark.parametrize("K,N", [(23, 64), (14, 64), (59, 64), (6, 32)])
def test_point_embed(device, K, N):
    """sfx_point_embed (the PTv3 embedding Linear -> eval BatchNorm -> GELU on the VALU, strided input rows as the
    head buffer holds them) vs torch fp64: rel L2 <= 1e-6."""
    g = torch.Generator().manual_seed(K)
    n = 4099
    buf = torch.randn(n, 160, generator=g)
    x = buf[:, 96:96 + K]
    w, b = torch.randn(N, K, generator=g) * 0.3, torch.randn(N, generator=g)
    sc, sh = torch.rand(N, generator=g) + 0.5, torch.randn(N, generator=g)
    bd = buf.to(device)
    y = ops.point_embed(bd[:, 96:96 + K], w.to(device), b.to(device), sc.to(device), sh.to(device))
    ref = torch.nn.functional.gelu((x.double() @ w.double().T + b.double()) * sc.double() + sh.double())
    assert rel_l2(y.cpu().double(), ref) < 1e-6


@pytest.mark.parametrize("sh", [1, 0, 3])
def test_fused_heads(device, sh):
    """sfx_heads (the six output MLPs + tanh + residual in one launch, csrc/heads.hip) vs the fp64 oracle heads
    (feature_predictor.py:201-235 restated in ptv3_ref.heads_forward) and vs the unfused GEMM chain: the refined
    residual within rel L2 2e-6; SH0 (5 heads, Cin 14), SH1 (Cin 23) and SH3 (Cin 59: input K padded to 160,
    a 45-wide output head); rows of very different magnitude; a row count not a multiple of 256."""
    from splatformer_amd.feature_predictor import FeaturePredictor
    torch.manual_seed(sh)
    fp = FeaturePredictor(sh_degree=sh, zeroinit=False)
    sd = {k: v.detach().double() for k, v in fp.state_dict().items()}
    fp = fp.to(device)
    cb, cin = 96, fp.gs_features_dim
    n = 5001
    g = torch.Generator().manual_seed(sh + 10)
    h0 = torch.zeros(n, (cb + cin + 3) // 4 * 4)
    h0[:, :cb + cin] = torch.randn(n, cb + cin, generator=g) * torch.exp2(torch.randint(-6, 7, (n, 1), generator=g).float())
    st, pr, ocols, out_dim = fp._fused_heads()
    n_tanh = 3
    y = ops.heads(h0.to(device), fp.head_in, cb, out_dim, n_tanh, ocols, st, pr).cpu()
    feat = h0[:, cb:cb + cin].double()
    in_gs, c = {}, 0
    for f in fp.output_features:
        w = fp.ch[f]
        in_gs[f] = feat[:, c:c + w].reshape(n, -1, 3) if f == "features_rest" else feat[:, c:c + w]
        c += w
    ref = ptv3_ref.heads_forward(sd, h0[:, :cb].double(), feat, in_gs, sh_degree=sh)
    rp = torch.cat([ref[f].reshape(n, -1) for f in fp.output_features], 1)
    err = rel_l2(y.double() - feat, rp - feat)
    assert err < 2e-6, err
    prev = ops.HEADS_FUSED
    ops.HEADS_FUSED = False
    try:
        w1, b1, mids, wl, bl, _ = fp._packed_heads()
        x = h0.to(device)[:, :w1.shape[1]]
        hh = ops.linear(x.contiguous(), w1, b1, act=ops.ACT_RELU)
        for wm, bm in mids:
            hh = ops.grouped_linear(hh, wm, bm, len(fp.output_features), act=ops.ACT_RELU)
        yu = ops.linear(hh, wl, bl, act=ops.ACT_TANH, act_ncols=n_tanh,
                        residual=h0.to(device)[:, cb:cb + cin].contiguous()).cpu()
    finally:
        ops.HEADS_FUSED = prev
    assert rel_l2(y.double() - feat, yu.double() - feat) < 4e-6


def test_subm_neighbors_duplicates_lowest_index(device):
    grid = torch.tensor([[5, 5, 5], [5, 5, 5], [6, 5, 5], [5, 5, 5], [0, 0, 0]], dtype=torch.int32)
    nbr = ops.subm_neighbors(grid.to(device), None, with_pairs=False).nbr.cpu()
    ref = ptv3_ref.subm_neighbors(grid, torch.zeros(5, dtype=torch.int64))
    assert torch.equal(nbr.long(), ref)
    assert nbr[3, 13] == 0 and nbr[0, 22] == 2  # centre -> lowest duplicate; +x neighbour
    assert (nbr[4, :13] == -1).all()  # negative coordinates never match


@pytest.mark.parametrize("dup", [False, True])
def test_serialization_exact(device, dup):
    s = make_scene(6000, 1, seed=7, unique_voxels=not dup)
    grid = torch.floor(s["means"] * 384).int()
    depth = int(grid.max()).bit_length()
    codes, order, inverse = ops.serialize(grid.to(device), None, depth, 3 * depth, ptv3_ref.ORDERS)
    c_ref, o_ref, i_ref, _ = serialize_ref.serialization(grid.numpy(), np.zeros(grid.shape[0], np.int64),
                                                         ptv3_ref.ORDERS, None)
    assert np.array_equal(codes.cpu().numpy(), c_ref)
    assert np.array_equal(order.cpu().numpy(), o_ref)
    assert np.array_equal(inverse.cpu().numpy(), i_ref)


def test_serialization_batched(device):
    s = make_scene(3000, 1, seed=8)
    grid = torch.floor(s["means"] * 384).int()
    offsets = torch.tensor([1000, 2200, 3000])
    batch = torch.repeat_interleave(torch.arange(3), torch.diff(offsets, prepend=torch.tensor([0])))
    depth = int(grid.max()).bit_length()
    cb = 3 * depth + 2
    codes, order, inverse = ops.serialize(grid.to(device), batch.int().to(device), depth, cb, ptv3_ref.ORDERS)
    c_ref, o_ref, i_ref, _ = serialize_ref.serialization(grid.numpy(), batch.numpy(), ptv3_ref.ORDERS, None)
    assert np.array_equal(codes.cpu().numpy(), c_ref)
    assert np.array_equal(order.cpu().numpy(), o_ref)
    assert np.array_equal(inverse.cpu().numpy(), i_ref)


@pytest.mark.parametrize("stride,B,perm,res", [(2, 1, [0, 1, 2, 3], 384), (2, 3, [2, 0, 3, 1], 384),
                                              (4, 2, [3, 2, 1, 0], 384), (2, 1, [1, 3, 0, 2], 1)])
def test_pooling_geometry_exact(device, stride, B, perm, res):
    """Sort-free SerializedPooling geometry vs the reference's integer math (pointtransformer_v3.py:290-299 ->
    Pointcept SerializedPooling: torch.unique(code[0] >> 3pd), stable sort(cluster), argsort of the pooled
    codes): clusters, CSR pointers, pooled codes / orders / inverses / grid / batch bit-exact; the members of a
    cluster as a set (listed in row0 serialized order here, index order in the reference); pooled coords
    (an fp32 mean of the same members in that order) to 1e-6."""
    from splatformer_amd.ptv3 import Point, SerializedPooling
    s = make_scene(5000, 1, seed=11, unique_voxels=False)
    grid = torch.floor(s["means"] * res).int()
    n = grid.shape[0]
    cuts = [0] + sorted(torch.randperm(n - 1, generator=torch.Generator().manual_seed(3))[:B - 1].add(1).tolist()) \
        + [n]
    batch = torch.repeat_interleave(torch.arange(B), torch.tensor(np.diff(cuts)))
    depth = int(grid.max()).bit_length()
    cb = 3 * depth + max(0, (B - 1).bit_length())
    bt = batch.int().to(device) if B > 1 else None
    codes, order, inverse = ops.serialize(grid.to(device), bt, depth, cb, ptv3_ref.ORDERS)
    pt = Point(coord=s["means"].to(device), grid_coord=grid.to(device), offset=cuts[1:], codes_phys=codes,
               order_phys=order, inverse_phys=inverse, order_type=list(perm), serialized_depth=depth, code_bits=cb)
    if bt is not None:
        pt.batch = bt
    new, sidx, idx_ptr, m = SerializedPooling(8, 8, stride=stride, norm_layer=torch.nn.BatchNorm1d,
                                                  act_layer=torch.nn.GELU).geometry(pt, [0, 1, 2, 3])

    # the reference's integer math on the oracle's serialization, rows in logical (permuted) order
    c_ref, _, _, _ = serialize_ref.serialization(grid.numpy(), batch.numpy(), ptv3_ref.ORDERS, None)
    code = torch.from_numpy(c_ref)[perm]
    pd = (stride - 1).bit_length()
    if pd > depth:
        pd = 0
    code = code >> 3 * pd
    _, cluster, counts = torch.unique(code[0], sorted=True, return_inverse=True, return_counts=True)
    indices = torch.sort(cluster, stable=True).indices
    ptr_ref = torch.cat([counts.new_zeros(1), torch.cumsum(counts, 0)])
    head = indices[ptr_ref[:-1]]
    code_h = code[:, head]
    order_ref = torch.argsort(code_h, stable=True)
    inv_ref = torch.zeros_like(order_ref).scatter_(1, order_ref, torch.arange(code_h.shape[1]).repeat(4, 1))

    assert m == len(counts)
    assert torch.equal(new.pooling_inverse.cpu().long(), cluster)
    assert torch.equal(idx_ptr.cpu().long(), ptr_ref)
    rows = new.order_type  # logical -> physical rows of the pooled point
    assert torch.equal(new.codes_phys.cpu()[rows], code_h)
    assert torch.equal(new.order_phys.cpu().long()[rows], order_ref)
    assert torch.equal(new.inverse_phys.cpu().long()[rows], inv_ref)
    assert torch.equal(new.grid_coord.cpu(), grid[head] >> pd)
    if B > 1:
        assert torch.equal(new.batch.cpu().long(), batch[head])
        assert new.offset == torch.cumsum(torch.bincount(batch[head]), 0).tolist()
    seg = torch.repeat_interleave(torch.arange(m), counts)
    key = seg * n + sidx.cpu().long()
    assert torch.equal(torch.sort(key).values, seg * n + indices)  # same members per cluster
    mean = torch.zeros(m, 3, dtype=torch.float64).index_add_(0, seg, s["means"][indices].double()) / counts[:, None]
    assert torch.allclose(new.coord.cpu().double(), mean, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("n", [1, 1000, 100_003])
def test_pool_run_counts(device, n):
    """sfx_pool_run_counts (every pooling's cluster count in one launch) == the run counts of code >> shift along
    the serialized row, for 1..9 shifts (9: two launches)."""
    g = torch.Generator().manual_seed(n)
    codes = torch.randint(0, 1 << 40, (1, n), generator=g, dtype=torch.int64) >> torch.randint(0, 30, (1, n),
                                                                                              generator=g)
    order = torch.randperm(n, generator=g).int()
    shifts = [0, 3, 6, 9, 12, 21, 27, 33, 39]
    c = codes[0][order.long()]
    ref = [int(1 + ((c[1:] >> s) != (c[:-1] >> s)).sum()) if n else 0 for s in shifts]
    for k in (1, 4, 9):
        got = ops.pool_counts_begin(codes.to(device), order[None].to(device), shifts[:k]).get()
        assert got == ref[:k]


@pytest.mark.parametrize("terms", ["bf16x3", "fp16x2"])
@pytest.mark.parametrize("n,heads,C", [(1000, 2, 64), (777, 4, 96), (300, 8, 128), (100, 2, 32)])
def test_window_attention_vs_reference_padding(device, n, heads, C, terms):
    """Window table == Pointcept get_padding_and_inverse duplication semantics (incl. K = n < 128); both MFMA
    term forms (fp16x2 needs an amax slot bounding |qkv|: here measured, and 8x loose)."""
    g = torch.Generator().manual_seed(n)
    qkv = torch.randn(n, 3 * C, generator=g) * (1e-3 if terms == "fp16x2" else 1.0)
    order = torch.randperm(n, generator=g)
    inverse = torch.empty_like(order)
    inverse[order] = torch.arange(n)
    offset = torch.tensor([n])
    K = min(n, 128)
    pad, unpad = ptv3_ref.get_padding_and_inverse(offset, K)
    o = order[pad]
    inv = unpad[inverse]
    q, k, v = qkv[o].reshape(-1, K, 3, heads, C // heads).permute(2, 0, 3, 1, 4).unbind(0)
    att = torch.softmax((q * (C // heads) ** -0.5) @ k.transpose(-2, -1), -1)
    ref = (att @ v).transpose(1, 2).reshape(-1, C)[inv]
    tab = ops.window_table([n], K)
    win = torch.tensor(tab, dtype=torch.int32).to(device)
    slot = None
    qd = qkv.to(device)
    if terms == "fp16x2":
        slot = ops.new_amax(qd.device)
        big = qd * 8  # a loose bound must do as well as the exact one
        from splatformer_amd._lib import call, ptr, stream
        call("sfx_amax_f32", n, 3 * C, ptr(big), 3 * C, slot[0], slot[1], stream())
    out = ops.window_attention(qd, order.int().to(device), win, len(tab), K, heads, C, qkv_amax=slot)
    assert rel_l2(out.cpu(), ref) < 2e-6


@pytest.mark.parametrize("n,heads,C", [(1000, 2, 64), (777, 4, 96), (300, 8, 128), (3000, 16, 256), (100, 16, 256),
                                       (129, 4, 96), (37_759, 16, 256), (100_000, 2, 64)])
def test_window_attention_proj(device, n, heads, C):
    """Fused attention + proj + residual (attn_proj.hip: x2 = x1 + proj(attn(qkv)), calflops.py:51-69) vs the fp64
    reference of the Pointcept padding semantics (as test_window_attention_vs_reference_padding) followed by the
    Linear and the residual add: ragged last windows, K = n < 128, a window of 129 points, the config-B stage
    shapes; fp16x2 terms from an 8x loose qkv bound.  Also within fp32 rounding of the unfused HIP path."""
    g = torch.Generator().manual_seed(n + C)
    qkv = torch.randn(n, 3 * C, generator=g) * 0.5
    x1 = torch.randn(n, C, generator=g)
    lin = torch.nn.Linear(C, C)
    with torch.no_grad():
        lin.weight.copy_(torch.randn(C, C, generator=g) * C ** -0.5)
        lin.bias.copy_(torch.randn(C, generator=g) * 0.1)
    order = torch.randperm(n, generator=g)
    inverse = torch.empty_like(order)
    inverse[order] = torch.arange(n)
    K = min(n, 128)
    pad, unpad = ptv3_ref.get_padding_and_inverse(torch.tensor([n]), K)
    q, k, v = qkv.double()[order[pad]].reshape(-1, K, 3, heads, C // heads).permute(2, 0, 3, 1, 4).unbind(0)
    att = torch.softmax((q * (C // heads) ** -0.5) @ k.transpose(-2, -1), -1)
    a = (att @ v).transpose(1, 2).reshape(-1, C)[unpad[inverse]]
    ref = x1.double() + a @ lin.weight.double().T + lin.bias.double()
    tab = ops.window_table([n], K)
    win = torch.tensor(tab, dtype=torch.int32).to(device)
    qd, od = qkv.to(device), order.int().to(device)
    lin = lin.to(device)
    slot = ops.new_amax(qd.device)
    big = qd * 8
    from splatformer_amd._lib import call, ptr, stream
    call("sfx_amax_f32", n, 3 * C, ptr(big), 3 * C, slot[0], slot[1], stream())
    x2 = ops.window_attention_proj(qd, od, win, len(tab), K, heads, C, lin, x1.to(device), slot)
    e = rel_l2(x2.cpu().double() - x1.double(), ref - x1.double())
    unf = ops.linear(ops.window_attention(qd, od, win, len(tab), K, heads, C, qkv_amax=slot), lin.weight, lin.bias,
                     residual=x1.to(device))
    e_unf = rel_l2(unf.cpu().double() - x1.double(), ref - x1.double())
    print(f"\n[attn+proj n={n} C={C}] branch rel L2 vs fp64: fused {e:.2e}, unfused {e_unf:.2e}")
    assert e < 2e-6 and e <= 2 * e_unf + 1e-7


@pytest.mark.parametrize("n,heads,C", [(100_000, 2, 64), (90_434, 4, 96), (37_759, 16, 256), (14_764, 32, 512),
                                       (3000, 4, 96), (77, 2, 64)])
def test_window_attention_seq_bitwise(device, n, heads, C, monkeypatch):
    """The pipelined attention (window_attn_seq_kernel: consecutive (window, head) items per workgroup, the next
    item's gathers in flight during the current one's MFMAs) equals the one-item-per-workgroup kernel bit for bit
    (same arithmetic, same term order) at the config-B stage shapes, a ragged last window and K = n < 128."""
    g = torch.Generator().manual_seed(n + heads)
    qkv = (torch.randn(n, 3 * C, generator=g) * 0.3).to(device)
    order = torch.randperm(n, generator=g).int().to(device)
    K = min(n, 128)
    tab = ops.window_table([n], K)
    win = torch.tensor(tab, dtype=torch.int32).to(device)
    slot = ops.new_amax(qkv.device)
    from splatformer_amd._lib import call, ptr, stream
    call("sfx_amax_f32", n, 3 * C, ptr(qkv), 3 * C, slot[0], slot[1], stream())
    monkeypatch.setenv("SFX_ATTN_SEQ", "1")
    a = ops.window_attention(qkv, order, win, len(tab), K, heads, C, qkv_amax=slot)
    monkeypatch.setenv("SFX_ATTN_SEQ", "0")
    b = ops.window_attention(qkv, order, win, len(tab), K, heads, C, qkv_amax=slot)
    assert torch.equal(a, b)


@pytest.mark.parametrize("terms", ["bf16x3", "fp16x2"])
@pytest.mark.parametrize("K", [1024, 256])
@pytest.mark.parametrize("heads,C", [(2, 32), (4, 96), (8, 256)])
def test_window_attention_flash_varlen(device, K, heads, C, terms):
    """enable_flash=True windows (pointtransformer_v3.py:121-123, K = 1024): batches of n < K (one n-key window),
    n == K, ragged n > K (last window padded with the preceding points) and n = 2K, one launch; vs the oracle's
    cu_seqlens restatement in fp64 (online softmax over 128-key blocks vs one softmax: order of summation only).
    Both MFMA term forms (fp16x2 from an 8x loose amax slot)."""
    counts = [700, K, 2 * K + 333, 2 * K, 5, 1]
    n = sum(counts)
    offset = torch.tensor(counts).cumsum(0)
    g = torch.Generator().manual_seed(K + C)
    qkv = torch.randn(n, 3 * C, generator=g, dtype=torch.float64) * 2
    batch = torch.repeat_interleave(torch.arange(len(counts)), torch.tensor(counts))
    order = torch.cat([torch.randperm(c, generator=g) + (int(offset[i]) - c) for i, c in enumerate(counts)])
    inverse = torch.empty_like(order)
    inverse[order] = torch.arange(n)
    point = ptv3_ref.Point(offset=offset, serialized_order=order[None], serialized_inverse=inverse[None], batch=batch)
    ref = ptv3_ref.serialized_attention_flash(qkv, point, C, heads, K, 0)
    tab = ops.window_table_varlen_np(offset.tolist(), K)
    win3 = torch.from_numpy(tab).to(device)
    qd = qkv.float().to(device)
    slot = None
    if terms == "fp16x2":
        slot = ops.new_amax(qd.device)
        big = qd * 8  # a loose bound must do as well as the exact one
        from splatformer_amd._lib import call, ptr, stream
        call("sfx_amax_f32", n, 3 * C, ptr(big), 3 * C, slot[0], slot[1], stream())
    out = ops.window_attention_varlen(qd, order.int().to(device), win3, tab.shape[0], K, heads, C, qkv_amax=slot)
    assert rel_l2(out.cpu(), ref) < 2e-6
    # every point written exactly once (no stale rows): a NaN-filled output buffer comes back NaN-free
    out2 = torch.full((n, C), float("nan"), device=device)
    ops.window_attention_varlen(qd, order.int().to(device), win3, tab.shape[0], K, heads, C, out=out2,
                                qkv_amax=slot)
    assert torch.equal(out2.cpu(), out.cpu())


def test_layernorm_ops(device):
    g = torch.Generator().manual_seed(2)
    for C in (64, 96, 128, 256, 512, 48):  # vectorised row-group kernels + the generic fallback (48)
        x = torch.randn(777, C, generator=g) * 3 + 1
        t = torch.randn(777, C, generator=g)
        ga, be = torch.randn(C, generator=g), torch.randn(C, generator=g)
        g1, b1 = torch.randn(C, generator=g), torch.randn(C, generator=g)
        y = ops.layernorm(x.to(device), ga.to(device), be.to(device), 1e-5).cpu()
        ref = torch.nn.functional.layer_norm(x, (C,), ga, be, 1e-5)
        assert rel_l2(y, ref) < 1e-6
        xo, h = ops.cpe_residual_ln(t.to(device), x.to(device), ga.to(device), be.to(device), g1.to(device),
                                    b1.to(device), 1e-5)
        xr = x + torch.nn.functional.layer_norm(t, (C,), ga, be, 1e-5)
        hr = torch.nn.functional.layer_norm(xr, (C,), g1, b1, 1e-5)
        assert rel_l2(xo.cpu(), xr) < 1e-6 and rel_l2(h.cpu(), hr) < 1e-6


# ---- whole refiner ---------------------------------------------------------------
def _randomize(model: torch.nn.Module, seed: int):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, torch.nn.BatchNorm1d):
                m.running_mean.copy_(torch.randn(m.num_features, generator=g) * 0.1)
                m.running_var.copy_(torch.rand(m.num_features, generator=g) + 0.5)
                m.weight.copy_(torch.rand(m.num_features, generator=g) + 0.5)
                m.bias.copy_(torch.randn(m.num_features, generator=g) * 0.1)
            if isinstance(m, torch.nn.LayerNorm):
                m.weight.copy_(torch.rand(m.normalized_shape, generator=g) + 0.5)
                m.bias.copy_(torch.randn(m.normalized_shape, generator=g) * 0.1)


def _model(seed=0, **bk):
    torch.manual_seed(seed)
    m = FeaturePredictor(sh_degree=1, zeroinit=False, backbone_kwargs=bk)
    _randomize(m, seed + 1)
    return m.eval()


@pytest.mark.parametrize("n,unique,bk", [
    (3000, True, {}),
    (5000, False, {}),
    (2000, True, dict(enc_depths=(1, 1, 1, 1, 1), dec_depths=(1, 1, 1, 1))),  # config A shape (depth 1)
    (6000, False, dict(enable_flash=True)),  # K = 1024 windows (pointtransformer_v3.py:121-123)
    (3000, False, dict(enc_dim=32)),  # enc_channels (32, 64, ...) (pointtransformer_v3.py:113): C=32 stage 0
])
def test_feature_predictor_matches_oracle(device, n, unique, bk):
    model = _model(3, **bk)
    cfg = ptv3_ref.PTv3Config(**{k: v for k, v in bk.items() if k != "enc_dim"})
    if bk.get("enc_dim") == 32:
        cfg.enc_channels = (32, 64, 128, 256, 512)
    if cfg.enable_flash:
        cfg.patch_size = 1024
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    model = model.to(device)
    s = make_scene(n, 1, seed=n, unique_voxels=unique)
    sd_in = to_device(s, device)
    torch.manual_seed(123)
    out = model([sd_in], [0])[0]
    perms = model.backbone.backbone.last_perms
    assert len(perms) == 5
    ref, point = ptv3_ref.feature_predictor_forward(sd, cfg, s, perms)
    for k in ["means", "scales", "opacities", "quats", "features_dc", "features_rest"]:
        got = out[k].cpu()
        assert got.shape == ref[k].shape, k
        err = rel_l2(got - s[k], ref[k] - s[k])  # error relative to the predicted residual
        assert err < 1e-5, f"{k}: rel L2 of residual {err}"


def test_backbone_feature_l2(device):
    model = _model(5)
    cfg = ptv3_ref.PTv3Config()
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    model = model.to(device)
    s = make_scene(4000, 1, seed=11, unique_voxels=True)
    data = ptv3_ref.batchify(s)
    perms = [[1, 0, 3, 2], [2, 3, 0, 1], [0, 1, 2, 3], [3, 2, 1, 0], [1, 3, 0, 2]]
    dd = {k: (v.to(device) if isinstance(v, torch.Tensor) else v) for k, v in data.items()}
    p = model.backbone(dd, perms=perms)
    ref = ptv3_ref.ptv3_forward(sd, cfg, data, perms, prefix="backbone.backbone.")
    assert rel_l2(p.feat.cpu(), ref.feat) < 1e-5


@pytest.mark.parametrize("cfg", list(range(ops.GEMM_NUM_CONFIGS)))
def test_gemm_every_tile_config(device, cfg):
    """Every tile configuration (incl. the eight-wave ping-pong tiles) and Stream-K on/off, for dense,
    gathered (one segment) and offset-major pair (SubM conv) launches, against fp64 products."""
    g = torch.Generator().manual_seed(cfg)
    n, C = 6000, 96
    s = make_scene(n, 1, seed=5, unique_voxels=True)
    grid = torch.floor(s["means"] * 384).int()
    nbr_ref = ptv3_ref.subm_neighbors(grid, torch.zeros(grid.shape[0], dtype=torch.int64))
    smap = ops.subm_neighbors(grid.to(device), None)
    try:
        for sk in (0, 1):
            ops.gemm_force_config(cfg, sk)
            for (M, N, K) in [(3001, 200, 64), (2500, 136, 544), (777, 520, 1024)]:
                x = torch.randn(M, K, generator=g)
                w = torch.randn(N, K, generator=g) / K ** 0.5
                b = torch.randn(N, generator=g)
                res = torch.randn(M, N, generator=g)
                ref = x.double() @ w.double().T + b.double() + res.double()
                y = ops.linear(x.to(device), w.to(device), b.to(device), residual=res.to(device))
                assert rel_l2(y.cpu(), ref) < 2e-6, (cfg, sk, M, N, K)
                yg = torch.nn.functional.gelu(x @ w.T + b)
                y2 = ops.linear(x.to(device), w.to(device), b.to(device), act=ops.ACT_GELU)
                assert rel_l2(y2.cpu(), yg) < 2e-6, (cfg, sk, M, N, K, "gelu")
            for cin in (C, 256):
                xx = torch.randn(grid.shape[0], cin, generator=g)
                ww = torch.randn(cin, 3, 3, 3, cin, generator=g) * 0.05
                bb = torch.randn(cin, generator=g)
                ref2 = ptv3_ref.subm_conv(xx, nbr_ref, ww, bb)
                y3 = ops.subm_conv(xx.to(device), smap, ww.to(device), bb.to(device))
                assert rel_l2(y3.cpu(), ref2) < 2e-6, (cfg, sk, cin, "conv")
    finally:
        ops.gemm_force_config(-1, -1)


def test_cached_bounds_survive_amax_ring_wrap(device):
    """Cached weight / LayerNorm bounds live in their own slots: after more than the ring's worth of producer
    launches (each publishing max |Y| into the next ring slot under a newer tag, as later forwards do) a second
    forward of the same model gives the same outputs (a cached bound in a recycled ring slot read
    0 or a too-small bound once a newer producer had written there)."""
    model = _model(9).to(device)
    s = to_device(make_scene(3000, 1, seed=4, unique_voxels=True), device)
    perms = [[0, 1, 2, 3]] * 5
    out1 = {k: v.clone() for k, v in model([s], [0], perms=perms)[0].items()}
    x = torch.full((64, 64), 1e3, device=device)
    w = torch.full((64, 64), 1e3, device=device)
    for _ in range(ops._AMAX_RING + 64):  # every ring slot rewritten with a newer tag and a large maximum
        ops.linear(x, w, None, y_amax=True)
    out2 = model([s], [0], perms=perms)[0]
    for k in out1:  # equal up to the SubM pair launch's float-atomic summation order
        assert torch.isfinite(out2[k]).all(), k
        assert rel_l2(out2[k].cpu() - s[k].cpu(), out1[k].cpu() - s[k].cpu()) < 1e-6, k
