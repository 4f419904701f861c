"""Oracle render glue vs golden vectors captured from the reference's own gs_utils.py
(tests/golden/make_golden.py).  Pins utils/gs_utils.py:31-95 argument semantics."""
import os

import numpy as np
import pytest
import torch

from oracle import gsplat_ref, render_ref

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "render_glue.npz")


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD))


@pytest.mark.parametrize("deg", [0, 1, 3])
def test_glue_args_match_reference(gold, deg):
    p = f"deg{deg}_"
    s = {k[len(p) + 3:]: torch.from_numpy(v) for k, v in gold.items() if k.startswith(p + "in_")}
    c2w = torch.from_numpy(gold[p + "c2w"])
    a = render_ref.glue_args(s, c2w)
    np.testing.assert_array_equal(a["viewmat"].numpy(), gold[p + "viewmat"])
    np.testing.assert_array_equal(a["scales"].numpy(), gold[p + "scales"])
    np.testing.assert_array_equal(a["quats"].numpy(), gold[p + "quats"])
    np.testing.assert_array_equal(a["opacities"].numpy(), gold[p + "opacity"])
    np.testing.assert_allclose(a["rgbs"].numpy(), gold[p + "colors"], rtol=0, atol=0)
    sc = gold[p + "proj_scalars"]
    assert sc[0] == 1 and sc[7] == 16  # glob_scale=1, BLOCK_WIDTH=16 (gs_utils.py:12, :85)
    intr = gold[p + "intr"]
    assert sc[5] == intr[5] and sc[6] == intr[4]  # H, W from height/width
    if deg > 0:
        assert int(gold[p + "sh_deg"]) == deg
        np.testing.assert_array_equal(a["viewdirs"].numpy(), gold[p + "sh_viewdirs"])
        np.testing.assert_array_equal(a["colors"].numpy(), gold[p + "sh_coeffs"])


def test_nan_quaternion_patched(gold):
    q = gold["deg1_quats"]
    np.testing.assert_array_equal(q[5], np.array([0, 0, 0, 1], dtype=np.float32))
    assert np.isfinite(q).all()


def test_metrics_oracle_matches_reference_golden():
    """oracle/metrics_ref.py (psnr, ssim) against outputs of the reference's own utils/metrics.py."""
    from oracle import metrics_ref
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "metrics.npz"))
    for i in range(2):
        a, b = torch.from_numpy(d[f"b{i}_img1"]), torch.from_numpy(d[f"b{i}_img2"])
        np.testing.assert_array_equal(metrics_ref.ssim(a, b, 11, size_average=False).numpy(), d[f"b{i}_ssim"])
        np.testing.assert_array_equal(metrics_ref.psnr(a, b).numpy(), d[f"b{i}_psnr"])


@pytest.mark.parametrize("deg", [0, 1, 3])
def test_canonical_glue_within_ulps_of_reference_ops(gold, deg):
    """The canonical glue arithmetic (float64 exp/sigmoid rounded once, left-to-right norms; the HIP eval
    path's) is within 2 ulp of the reference-op form pinned above."""
    p = f"deg{deg}_"
    s = {k[len(p) + 3:]: torch.from_numpy(v) for k, v in gold.items() if k.startswith(p + "in_")}
    c2w = torch.from_numpy(gold[p + "c2w"])
    a = render_ref.glue_args(s, c2w)
    c = render_ref.glue_args(s, c2w, canonical=True)
    for k in ["viewmat", "scales", "quats", "opacities", "rgbs"]:
        x, y = a[k].numpy(), c[k].numpy()
        ulp = np.spacing(np.maximum(np.abs(x), np.abs(y)).astype(np.float32))
        if k == "viewmat":  # -R^T t cancels: rounding is relative to the summands' magnitude
            ulp = np.maximum(ulp, np.spacing(np.float32(np.abs(c2w.numpy()).max())))
        assert np.all(np.abs(x - y) <= 2 * ulp + 1e-30), k


def test_vectorised_intersections_match_loop():
    """map_gaussian_to_intersects (vectorised) == the per-Gaussian loop of gsplat's kernel."""
    from splatformer_amd.scenes import make_cameras, make_scene
    s = make_scene(3000, 1, seed=7)
    cams = make_cameras(200, 150, n_views=1)
    a = render_ref.glue_args(s, cams["camera_to_worlds"][0], canonical=True)
    xys, depths, radii, _, _, tiles, _ = gsplat_ref.project_gaussians(
        a["means"], a["scales"], 1.0, a["quats"], a["viewmat"], cams["fx"], cams["fy"], cams["cx"], cams["cy"], 150,
        200, 16)
    tx, ty = 13, 10
    cum = torch.cumsum(tiles, 0, dtype=torch.int32)
    keys, gids = gsplat_ref.map_gaussian_to_intersects(xys, depths, radii, cum, tx, ty, 16)
    x0, y0, x1, y1 = gsplat_ref.tile_bbox(xys, radii, tx, ty, 16)
    dbits = depths.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    k2, g2 = [], []
    for i in range(xys.shape[0]):
        if radii[i] <= 0:
            continue
        for yy in range(int(y0[i]), int(y1[i])):
            for xx in range(int(x0[i]), int(x1[i])):
                k2.append(((yy * tx + xx) << 32) | int(dbits[i]))
                g2.append(i)
    assert torch.equal(keys, torch.tensor(k2, dtype=torch.int64))
    assert torch.equal(gids, torch.tensor(g2, dtype=torch.int32))
