"""HIP render path (libsfx) vs the gsplat v0.1.11 CPU oracle on identical inputs.

Tolerances: the projection follows the oracle's canonical arithmetic (no
contraction, left-to-right sums, correctly rounded division/sqrt), so every
projection output -- integer and float -- is bit-exact; integer/index outputs
(radii, tile counts, sorted intersection ids, tile bins) bit-exact; images
within 2e-4 absolute and |dPSNR| <= 1e-4 dB on uint8-quantised renders
(BASELINE.json north_star).  Full-size workloads: tests/test_gpu_full.py.
"""
import math

import pytest
import torch

from oracle import gsplat_ref, render_ref
from splatformer_amd import gs_render, gsplat_compat
from splatformer_amd.scenes import make_cameras, make_scene, to_device

pytestmark = pytest.mark.gpu


def _scene(n, deg, seed):
    return make_scene(n, sh_degree=deg, seed=seed)


@pytest.mark.parametrize("deg", [0, 1, 2, 3, 4])
def test_sh_fwd_bwd(device, deg):
    n = 3000
    g = torch.Generator().manual_seed(deg)
    nb = (deg + 1) ** 2
    coeffs = torch.randn(n, nb + 1 if deg < 4 else nb, 3, generator=g)  # extra basis -> stride test
    dirs = torch.randn(n, 3, generator=g)
    ref = gsplat_ref.spherical_harmonics(deg, dirs, coeffs)
    c = coeffs.to(device).requires_grad_(True)
    out = gsplat_compat.spherical_harmonics(deg, dirs.to(device), c)
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-5, atol=5e-6)
    v = torch.randn(n, 3, generator=g)
    out.backward(v.to(device))
    refg = gsplat_ref.spherical_harmonics_bwd(deg, dirs, v, coeffs.shape[1])
    torch.testing.assert_close(c.grad.cpu(), refg, rtol=1e-5, atol=1e-6)


def _proj_inputs(n, seed, W=160, H=120):
    s = make_scene(n, 1, seed)
    cams = make_cameras(W, H, n_views=9)
    c2w = cams["camera_to_worlds"][seed % 9]
    a = render_ref.glue_args(s, c2w)
    return a, cams, W, H


@pytest.mark.parametrize("seed,n,W,H", [(0, 5000, 160, 120), (4, 5000, 160, 120), (8, 5000, 160, 120),
                                         (2, 100_000, 800, 800)])
def test_project_fwd(device, seed, n, W, H):
    """Every output bit-exact (round 1 tolerated max(2, n/2000) integer mismatches; 0 measured at 100k x 9
    views 800x800 before the canonical-arithmetic change, profiles/r02_proj_mismatch_before.json)."""
    a, cams, W, H = _proj_inputs(n, seed, W, H)
    args = (a["means"], a["scales"], 1.0, a["quats"], a["viewmat"], cams["fx"], cams["fy"], cams["cx"], cams["cy"], H,
            W, 16)
    ref = gsplat_ref.project_gaussians(*args)
    dev = [x.to(device) if isinstance(x, torch.Tensor) else x for x in args]
    out = gsplat_compat.project_gaussians(*dev)
    names = ["xys", "depths", "radii", "conics", "comp", "num_tiles_hit", "cov3d"]
    for nm, r, o in zip(names, ref, out):
        o = o.cpu()
        assert r.dtype == o.dtype and r.shape == o.shape, nm
        mism = (r != o).sum().item()
        assert mism == 0, f"{nm}: {mism} mismatches (max |d| {(r.double() - o.double()).abs().max().item():.3e})"


def test_scan_and_sort_exact(device):
    g = torch.Generator().manual_seed(3)
    for n in [1, 5, 2047, 2048, 2049, 100_000, 1_234_567]:
        keys = torch.randint(0, 1 << 44, (n,), generator=g, dtype=torch.int64)
        keys[::7] = keys[0]  # many ties -> stability matters
        vals = torch.randperm(n, generator=g).to(torch.int32)
        kd, vd = keys.to(device), vals.to(device)
        ko, vo = torch.empty_like(kd), torch.empty_like(vd)
        from splatformer_amd import _lib
        ws = _lib.workspace(_lib.fn("sfx_sort_workspace_bytes")(n), device)
        _lib.call("sfx_sort_pairs_u64", n, kd.data_ptr(), vd.data_ptr(), ko.data_ptr(), vo.data_ptr(), 0, 44,
                  ws.data_ptr(), ws.numel(), _lib.stream())
        ref = torch.sort(keys, stable=True)
        assert torch.equal(ko.cpu(), ref.values)
        assert torch.equal(vo.cpu(), vals[ref.indices])
        # argsort mode (vals NULL)
        _lib.call("sfx_sort_pairs_u64", n, kd.data_ptr(), None, ko.data_ptr(), vo.data_ptr(), 0, 44,
                  ws.data_ptr(), ws.numel(), _lib.stream())
        assert torch.equal(vo.cpu().long(), ref.indices)
        cnt = torch.randint(0, 9, (n,), generator=g, dtype=torch.int32)
        total, cum = gsplat_compat.compute_cumulative_intersects(cnt.to(device))
        assert total == int(cnt.sum())
        assert torch.equal(cum.cpu(), torch.cumsum(cnt, 0, dtype=torch.int32))


def test_lookback_scan_and_onesweep_sort_cases(device):
    """The single-pass scan and the radix sort's per-pass scans (decoupled look-back, ABI v11) on the cases their hand-off has to
    survive: thousands of tiles (long look-back chains, tiles finishing out of order), one workspace reused by
    back-to-back calls of different sizes without a host sync, exclusive and in-place scans, a bit range that
    does not start at 0, 64-bit keys using all passes, and negative values."""
    from splatformer_amd import _lib
    g = torch.Generator().manual_seed(11)
    ws = _lib.workspace(_lib.fn("sfx_scan_workspace_bytes")(6_000_000), device)
    outs = []
    for n, incl in [(6_000_000, 1), (4097, 0), (1, 0), (3_000_001, 0), (2048 * 37, 1)]:
        x = torch.randint(-5, 9, (n,), generator=g, dtype=torch.int32)
        xd = x.to(device)
        out = torch.empty_like(xd)
        tot = torch.zeros(1, device=device, dtype=torch.int32)
        _lib.call("sfx_scan_i32", n, xd.data_ptr(), out.data_ptr(), incl, ws.data_ptr(), ws.numel(), tot.data_ptr(),
                  _lib.stream())
        outs.append((x, incl, out, tot))
    for x, incl, out, tot in outs:  # checked after all launches: no sync between the reuses of `ws`
        ref = torch.cumsum(x, 0, dtype=torch.int32)
        if not incl:
            ref = ref - x
        assert torch.equal(out.cpu(), ref) and int(tot) == int(x.sum())
    x = torch.randint(0, 100, (777_777,), generator=g, dtype=torch.int32)
    xd = x.to(device)
    _lib.call("sfx_scan_i32", x.numel(), xd.data_ptr(), xd.data_ptr(), 1, ws.data_ptr(), ws.numel(), None,
              _lib.stream())  # in place
    assert torch.equal(xd.cpu(), torch.cumsum(x, 0, dtype=torch.int32))
    # more tiles than the stream's look-back area holds (65536 words): the area is reallocated, then a small scan
    # and a sort on the new one; totals written without a zeroed `total`
    for n in (2048 * 65536 + 3, 5000):
        x = torch.randint(0, 2, (n,), generator=g, dtype=torch.int32)
        xd = x.to(device)
        out = torch.empty_like(xd)
        tot = torch.full((1,), -7, device=device, dtype=torch.int32)
        wsn = _lib.workspace(_lib.fn("sfx_scan_workspace_bytes")(n), device)
        _lib.call("sfx_scan_i32", n, xd.data_ptr(), out.data_ptr(), 1, wsn.data_ptr(), wsn.numel(), tot.data_ptr(),
                  _lib.stream())
        assert torch.equal(out.cpu(), torch.cumsum(x, 0, dtype=torch.int32)) and int(tot) == int(x.sum()), n
        del xd, out
    for n, lo, hi in [(5_000_000, 0, 47), (300_000, 5, 61), (70_000, 0, 64)]:
        keys = torch.randint(-(1 << 62), 1 << 62, (n,), generator=g, dtype=torch.int64)
        keys[::3] = keys[1]
        if hi - lo < 64:
            keys &= (1 << hi) - 1
        kd = keys.to(device)
        ko, vo = torch.empty_like(kd), torch.empty(n, device=device, dtype=torch.int32)
        wss = _lib.workspace(_lib.fn("sfx_sort_workspace_bytes")(n), device)
        _lib.call("sfx_sort_pairs_u64", n, kd.data_ptr(), None, ko.data_ptr(), vo.data_ptr(), lo, hi,
                  wss.data_ptr(), wss.numel(), _lib.stream())
        ku = keys.cpu().numpy().view("uint64")
        sk = (ku >> lo) if hi == 64 else ((ku >> lo) & ((1 << (hi - lo)) - 1) if hi - lo < 64 else ku)
        import numpy as np
        order = np.argsort(sk, kind="stable")
        assert np.array_equal(vo.cpu().numpy(), order.astype(np.int32)), (n, lo, hi)
        assert np.array_equal(ko.cpu().numpy().view("uint64"), ku[order]), (n, lo, hi)
    # no look-back wait of any of these scans / passes reached the spin cap (ABI v12 counter); a
    # released area is reallocated by the next scan with a fresh counter
    assert _lib.fn("sfx_lookback_timeouts")(_lib.stream()) == 0
    _lib.call("sfx_lookback_release", _lib.stream())
    assert _lib.fn("sfx_lookback_timeouts")(_lib.stream()) == -1
    xd = torch.ones(5000, device=device, dtype=torch.int32)
    _lib.call("sfx_scan_i32", 5000, xd.data_ptr(), xd.data_ptr(), 1, None, 0, None, _lib.stream())
    assert int(xd[-1]) == 5000 and _lib.fn("sfx_lookback_timeouts")(_lib.stream()) == 0


def test_bin_and_sort_exact(device):
    a, cams, W, H = _proj_inputs(4000, 2)
    ref = gsplat_ref.project_gaussians(a["means"], a["scales"], 1.0, a["quats"], a["viewmat"], cams["fx"],
                                       cams["fy"], cams["cx"], cams["cy"], H, W, 16)
    xys, depths, radii, _, _, tiles, _ = ref
    tx, ty = (W + 15) // 16, (H + 15) // 16
    k_ref, g_ref, b_ref = gsplat_ref.bin_and_sort_gaussians(xys, depths, radii, tiles, tx, ty, 16)
    num, cum = gsplat_compat.compute_cumulative_intersects(tiles.to(device))
    assert num == k_ref.numel()
    _, _, ks, gs, bins = gsplat_compat.bin_and_sort_gaussians(xys.shape[0], num, xys.to(device), depths.to(device),
                                                              radii.to(device), cum, (tx, ty, 1), 16)
    assert torch.equal(ks.cpu(), k_ref)
    assert torch.equal(gs.cpu(), g_ref)
    assert torch.equal(bins.cpu(), b_ref)


def _psnr_u8(x, gt):
    return float(gsplat_ref.psnr_u8(x[None], gt[None]))


@pytest.mark.parametrize("deg,n,res", [(1, 4000, (128, 96)), (0, 2000, (64, 64)), (3, 3000, (100, 70))])
def test_render_fused_matches_oracle(device, deg, n, res):
    W, H = res
    s = _scene(n, deg, seed=deg + 20)
    cams = make_cameras(W, H, n_views=3)
    cams["background_color"] = torch.tensor([0.05, 0.1, 0.2])
    gt = torch.rand(H, W, 3, generator=torch.Generator().manual_seed(9))
    sd, cd = to_device(s, device), to_device(cams, device)
    for v in range(3):
        c2w = cams["camera_to_worlds"][v]
        rr, ar = render_ref.rasterize_gaussians_to_singleimg(s, c2w, **cams)
        with torch.no_grad():
            rh, ah = gs_render.rasterize_gaussians_to_singleimg(sd, cd["camera_to_worlds"][v], **cd)
        rh, ah = rh.cpu(), ah.cpu()
        assert rh.shape == (H, W, 3) and ah.shape == (H, W, 1)
        torch.testing.assert_close(rh, rr, rtol=0, atol=2e-4)
        torch.testing.assert_close(ah, ar, rtol=0, atol=2e-4)
        assert abs(_psnr_u8(rh, gt) - _psnr_u8(rr, gt)) <= 1e-4
        # mean abs error, and the PSNR between the two renders, far above quantisation
        assert (rh - rr).abs().mean() < 1e-6


def test_render_empty_and_culled(device):
    cams = make_cameras(32, 32, n_views=1)
    s = make_scene(50, 1, seed=1)
    s["means"] = s["means"] + 10.0  # far outside the frustum / behind: all culled
    sd, cd = to_device(s, device), to_device(cams, device)
    with torch.no_grad():
        rh, ah = gs_render.rasterize_gaussians_to_singleimg(sd, cd["camera_to_worlds"][0], **cd)
    rr, ar = render_ref.rasterize_gaussians_to_singleimg(s, cams["camera_to_worlds"][0], **cams)
    torch.testing.assert_close(rh.cpu(), rr)
    torch.testing.assert_close(ah.cpu(), ar)  # gsplat empty-branch: alpha == 1


def test_render_backward_matches_oracle(device):
    W, H = 96, 80
    s = _scene(1500, 1, seed=31)
    cams = make_cameras(W, H, n_views=2)
    c2w = cams["camera_to_worlds"][1]
    a = render_ref.glue_args(s, c2w)
    xys, depths, radii, conics, comp, tiles, cov3d = gsplat_ref.project_gaussians(
        a["means"], a["scales"], 1.0, a["quats"], a["viewmat"], cams["fx"], cams["fy"], cams["cx"], cams["cy"], H, W,
        16)
    bg = torch.tensor([0.3, 0.2, 0.1])
    g = torch.Generator().manual_seed(5)
    v_out = torch.randn(H, W, 3, generator=g)
    v_alpha = torch.randn(H, W, generator=g)
    # HIP forward+backward through the autograd Function
    t = lambda x: x.to(device).clone().requires_grad_(x.dtype == torch.float32)
    xd, cd_, rd, od = t(xys), t(conics), t(a["rgbs"]), t(a["opacities"])
    img, alpha = gsplat_compat.rasterize_gaussians(xd, depths.to(device), radii.to(device), cd_, tiles.to(device), rd,
                                                   od, H, W, 16, background=bg.to(device), return_alpha=True)
    (img * v_out.to(device)).sum().add_((alpha * v_alpha.to(device)).sum()).backward()
    # oracle backward on the oracle forward state
    tx, ty = (W + 15) // 16, (H + 15) // 16
    _, gids, bins = gsplat_ref.bin_and_sort_gaussians(xys, depths, radii, tiles, tx, ty, 16)
    _, fT, fidx = gsplat_ref.rasterize_forward(tx, ty, 16, H, W, gids, bins, xys, conics, a["rgbs"], a["opacities"],
                                               bg)
    # alpha = 1 - T -> dL/dalpha enters with the reference's sign convention
    rv = gsplat_ref.rasterize_backward(tx, ty, 16, H, W, gids, bins, xys, conics, a["rgbs"], a["opacities"], bg, fT,
                                       fidx, v_out, v_alpha)
    for nm, got, exp in zip(["v_xy", "v_conic", "v_rgb", "v_opacity"], [xd.grad, cd_.grad, rd.grad, od.grad], rv):
        got = got.cpu()
        scale = exp.abs().max().clamp_min(1e-6)
        err = (got - exp).abs().max() / scale
        assert err < 2e-4, f"{nm}: rel err {err}"


def test_project_backward_matches_oracle(device):
    a, cams, W, H = _proj_inputs(3000, 5)
    args = (a["means"], a["scales"], 1.0, a["quats"], a["viewmat"], cams["fx"], cams["fy"], cams["cx"], cams["cy"], H,
            W, 16)
    xys, depths, radii, conics, comp, tiles, cov3d = gsplat_ref.project_gaussians(*args)
    g = torch.Generator().manual_seed(1)
    n = xys.shape[0]
    vx, vc = torch.randn(n, 2, generator=g), torch.randn(n, 3, generator=g) * 1e-3
    vd, vco = torch.zeros(n), torch.zeros(n)
    ref = gsplat_ref.project_gaussians_backward(a["means"], a["scales"], 1.0, a["quats"], a["viewmat"], cams["fx"],
                                                cams["fy"], cov3d, radii, conics, comp, vx, vd, vc, vco)
    m = a["means"].to(device).requires_grad_(True)
    sc = a["scales"].to(device).requires_grad_(True)
    q = a["quats"].to(device).requires_grad_(True)
    out = gsplat_compat.project_gaussians(m, sc, 1.0, q, a["viewmat"].to(device), cams["fx"], cams["fy"], cams["cx"],
                                          cams["cy"], H, W, 16)
    (out[0] * vx.to(device)).sum().add_((out[3] * vc.to(device)).sum()).backward()
    for nm, got, exp in zip(["v_mean", "v_scale", "v_quat"], [m.grad, sc.grad, q.grad], ref):
        got = got.cpu()
        live = radii > 0
        scale = exp[live].abs().max().clamp_min(1e-6)
        err = ((got - exp)[live].abs().max() / scale).item()
        assert err < 1e-4, f"{nm}: rel err {err}"
        assert float(got[~live].abs().max() if (~live).any() else 0) == 0.0


def test_batched_views_equal_per_view(device):
    """rasterize_gaussians_to_multiimgs' batched eval path (one prep / sort / raster for all views) gives
    bit-identical images to rendering the views one by one, incl. gsplat's empty-view branch (alpha = 1)."""
    s = to_device(make_scene(20000, 1, seed=12), device)
    cams = make_cameras(160, 120, n_views=5)
    c2w = cams["camera_to_worlds"].clone()
    away = c2w[1].clone()
    away[:3, 3] = away[:3, 3] - 1000.0 * away[:3, 2]  # pushed past the scene, looking away: no intersection
    cams["camera_to_worlds"] = torch.cat([c2w, away[None]], 0)
    cams = to_device(cams, device)
    with torch.no_grad():
        rgbs, alphas = gs_render.rasterize_gaussians_to_multiimgs(s, cams)
        assert len(rgbs) == 6
        for v in range(6):
            r1, a1 = gs_render.rasterize_gaussians_to_singleimg(s, cams["camera_to_worlds"][v], **cams)
            assert torch.equal(rgbs[v], r1), v
            assert torch.equal(alphas[v], a1), v
    assert float(alphas[5].min()) == 1.0  # empty-branch quirk reproduced per view


def _render_both(sd, cams):
    """Eval render with and without exact contribution culling (ABI v9)."""
    cull0 = gs_render.RENDER_CULL
    try:
        gs_render.RENDER_CULL = True
        rc, ac, mc = gs_render.render_views_meta(sd, cams)
        gs_render.RENDER_CULL = False
        rf, af, mf = gs_render.render_views_meta(sd, cams)
    finally:
        gs_render.RENDER_CULL = cull0
    return (rc, ac, mc), (rf, af, mf)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_render_cull_bit_identical_adversarial(device, seed):
    """Culling near its thresholds: opacities around 1/255, needle-thin and near-degenerate (rho -> 1)
    conics, Gaussians sitting on tile and quadrant borders, image sizes that are not multiples of 16.  Images,
    alphas and final T must be bit-identical to the full gsplat list; the culled list must be shorter."""
    n = 6000
    g = torch.Generator().manual_seed(100 + seed)
    s = make_scene(n, 1, seed=seed)
    logit = lambda p: math.log(p / (1.0 - p))
    k = torch.randint(0, 4, (n,), generator=g)
    op = s["opacities"].clone()
    near = torch.tensor([logit(1 / 255.0)]) + 1e-4 * torch.randn(n, 1, generator=g)
    op[k == 0] = near[k == 0]  # opacity at the 1/255 threshold
    op[k == 1] = logit(0.999)
    s["opacities"] = op
    sc = s["scales"].clone()
    sc[k == 2, 0] = sc[k == 2, 0] + 3.0   # needles: one axis 20x, another 1/20
    sc[k == 2, 1] = sc[k == 2, 1] - 3.0
    s["scales"] = sc
    cams = make_cameras(200, 136, n_views=3)
    sd, cd = to_device(s, device), to_device(cams, device)
    with torch.no_grad():
        (rc, ac, mc), (rf, af, mf) = _render_both(sd, cd)
    torch.cuda.synchronize()
    assert mc["culled"] and not mf["culled"]
    assert mc["isect_sorted"].numel() < mf["isect_sorted"].numel()
    for v in range(3):
        assert torch.equal(rc[v], rf[v]), v
        assert torch.equal(ac[v], af[v]), v
        assert torch.equal(mc["final_Ts"][v], mf["final_Ts"][v]), v
    # every kept (tile, Gaussian) pair is one of gsplat's, in gsplat's order
    kf = zip((mf["isect_sorted"].cpu() >> 32).tolist(), mf["gids_sorted"].cpu().tolist())
    pos = {tg: i for i, tg in enumerate(kf)}
    p = [pos[tg] for tg in zip((mc["isect_sorted"].cpu() >> 32).tolist(), mc["gids_sorted"].cpu().tolist())]
    assert all(b > a for a, b in zip(p, p[1:]))


def test_render_cull_all_culled_view(device):
    """A view whose every gsplat intersection is culled (opacities below 1/255) renders background with alpha 0
    (gsplat's normal path), not the empty-list branch (alpha 1)."""
    s = make_scene(500, 1, seed=3)
    s["opacities"] = torch.full_like(s["opacities"], math.log((0.5 / 255) / (1 - 0.5 / 255)))
    cams = to_device(make_cameras(64, 48, n_views=2), device)
    sd = to_device(s, device)
    with torch.no_grad():
        (rc, ac, mc), (rf, af, mf) = _render_both(sd, cams)
    assert mf["isect_sorted"].numel() > 0
    for v in range(2):
        assert torch.equal(rc[v], rf[v]), v
        assert torch.equal(ac[v], af[v]), v
        assert float(ac[v].max()) == 0.0


def test_render_cull_training_grads_match_full(device):
    """Training render (autograd glue) over the culled list: forward images bit-identical to gsplat's full list,
    gradients of every Gaussian attribute equal up to float-atomic summation order (rel. 1e-5)."""
    from splatformer_amd import gsplat_compat
    s = to_device(make_scene(8000, 1, seed=21), device)
    cams = to_device(make_cameras(200, 152, n_views=2), device)
    res = {}
    cull0 = gsplat_compat.CULL
    try:
        for cull in (False, True):
            gsplat_compat.CULL = cull
            p = {k: v.clone().requires_grad_(True) for k, v in s.items()}
            rgbs, alphas = gs_render.rasterize_gaussians_to_multiimgs(p, cams)
            w = torch.linspace(0.5, 1.5, rgbs[0].numel(), device=device).reshape(rgbs[0].shape)
            loss = sum((r * w).sum() + 0.3 * a.sum() for r, a in zip(rgbs, alphas))
            loss.backward()
            res[cull] = ([r.detach() for r in rgbs], [a.detach() for a in alphas], {k: v.grad for k, v in p.items()})
    finally:
        gsplat_compat.CULL = cull0
    for v in range(2):
        assert torch.equal(res[True][0][v], res[False][0][v]), v
        assert torch.equal(res[True][1][v], res[False][1][v]), v
    for k, g_full in res[False][2].items():
        g = res[True][2][k]
        err = float((g - g_full).norm() / g_full.norm().clamp_min(1e-30))
        assert err <= 1e-5, f"grad {k}: rel {err:.3e}"
