"""Known-answer tests for the gsplat v0.1.11 CPU oracle (SURVEY.md §8(c) KATs 3-5)."""
import math

import torch

from oracle import gsplat_ref


def test_sh_degree0_is_c0_times_dc():
    c = torch.randn(10, 1, 3)
    d = torch.randn(10, 3)
    out = gsplat_ref.spherical_harmonics(0, d, c)
    torch.testing.assert_close(out, gsplat_ref.SH_C0 * c[:, 0], rtol=0, atol=0)


def test_sh_degree1_formula_and_renormalisation():
    c = torch.randn(7, 4, 3)
    d = torch.randn(7, 3) * 3.0
    out = gsplat_ref.spherical_harmonics(1, d, c)
    u = d / d.norm(dim=-1, keepdim=True)
    x, y, z = u[:, :1], u[:, 1:2], u[:, 2:3]
    exp = gsplat_ref.SH_C0 * c[:, 0] + gsplat_ref.SH_C1 * (-y * c[:, 1] + z * c[:, 2] - x * c[:, 3])
    torch.testing.assert_close(out, exp, rtol=1e-6, atol=1e-6)


def test_identity_camera_projection_center():
    means = torch.tensor([[0.1, -0.2, 2.0], [0.0, 0.0, 0.005]])
    scales = torch.full((2, 3), 0.01)
    quats = torch.tensor([[1.0, 0, 0, 0], [1.0, 0, 0, 0]])
    vm = torch.eye(4)[:3]
    fx, fy, cx, cy = 100.0, 120.0, 32.0, 24.0
    xys, depths, radii, conics, comp, tiles, cov3d = gsplat_ref.project_gaussians(
        means, scales, 1.0, quats, vm, fx, fy, cx, cy, 48, 64, 16)
    torch.testing.assert_close(xys[0], torch.tensor([fx * 0.1 / 2.0 + cx, fy * -0.2 / 2.0 + cy]), rtol=1e-5,
                               atol=1e-4)
    assert depths[0] == 2.0 and radii[0] > 0 and tiles[0] > 0
    # near-plane cull (z <= 0.01): every output zero
    assert radii[1] == 0 and tiles[1] == 0 and float(xys[1].abs().sum()) == 0.0
    # isotropic cov3d = s^2 I
    torch.testing.assert_close(cov3d[0], torch.tensor([1e-4, 0, 0, 1e-4, 0, 1e-4]), rtol=1e-5, atol=1e-9)


def test_single_gaussian_peak_pixel():
    """Isotropic Gaussian centred on a pixel centre: peak = min(0.999, o)*c + (1-alpha)*bg."""
    H = W = 32
    xys = torch.tensor([[16.5, 16.5]])
    conics = torch.tensor([[1 / 9.0, 0.0, 1 / 9.0]])
    radii = torch.tensor([9], dtype=torch.int32)
    depths = torch.tensor([1.0])
    tiles = torch.tensor([4], dtype=torch.int32)
    colors = torch.tensor([[0.2, 0.5, 0.9]])
    op = torch.tensor([[0.8]])
    bg = torch.tensor([0.1, 0.1, 0.1])
    img, alpha = gsplat_ref.rasterize_gaussians(xys, depths, radii, conics, tiles, colors, op, H, W, 16,
                                                background=bg, return_alpha=True)
    exp = 0.8 * colors[0] + 0.2 * bg
    torch.testing.assert_close(img[16, 16], exp, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(alpha[16, 16], torch.tensor(0.8), rtol=1e-6, atol=1e-6)
    # one pixel off-centre: alpha = o * exp(-0.5 * 1/9)
    a1 = 0.8 * math.exp(-0.5 / 9.0)
    torch.testing.assert_close(alpha[16, 17], torch.tensor(a1), rtol=1e-5, atol=1e-6)


def test_early_termination_excludes_saturating_gaussian():
    """T*(1-alpha) <= 1e-4 stops the pixel *before* adding that Gaussian (rasterize_forward)."""
    H = W = 16
    n = 3
    xys = torch.full((n, 2), 8.5)
    conics = torch.tensor([[1.0, 0.0, 1.0]] * n)
    radii = torch.full((n,), 3, dtype=torch.int32)
    depths = torch.tensor([1.0, 2.0, 3.0])
    tiles = torch.ones(n, dtype=torch.int32)
    colors = torch.tensor([[1.0, 0, 0], [0, 1.0, 0], [0, 0, 1.0]])
    op = torch.tensor([[0.999], [0.99], [0.5]])
    img, alpha = gsplat_ref.rasterize_gaussians(xys, depths, radii, conics, tiles, colors, op, H, W, 16,
                                                background=torch.zeros(3), return_alpha=True)
    # G0 alpha 0.999 -> T=1e-3; G1 alpha .99 -> nextT=1e-5 <= 1e-4 -> stop, G1 not added
    torch.testing.assert_close(img[8, 8], torch.tensor([0.999, 0.0, 0.0]), rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(alpha[8, 8], torch.tensor(0.999), rtol=1e-6, atol=1e-7)


def test_sort_key_tile_major_depth_minor():
    xys = torch.tensor([[5.0, 5.0], [5.0, 5.0], [20.0, 5.0]])
    depths = torch.tensor([2.0, 1.0, 0.5])
    radii = torch.tensor([1, 1, 1], dtype=torch.int32)
    tiles = torch.tensor([1, 1, 1], dtype=torch.int32)
    keys, gids, bins = gsplat_ref.bin_and_sort_gaussians(xys, depths, radii, tiles, 2, 1, 16)
    assert gids.tolist() == [1, 0, 2]
    assert bins.tolist() == [[0, 2], [2, 3]]


def test_psnr_uint8_truncation():
    a = torch.full((1, 4, 4, 3), 128.05 / 255)
    b = torch.full((1, 4, 4, 3), 128.95 / 255)  # both truncate to uint8 128
    assert torch.isinf(gsplat_ref.psnr_u8(a, b)).all()
