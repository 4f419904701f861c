"""CPU restatement of the reference render glue (utils/gs_utils.py:20-114).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Pinned by the golden
vectors in tests/golden/render_glue.npz, captured from the reference glue
itself (tests/golden/make_golden.py).
"""
from __future__ import annotations

import math

import torch

from . import gsplat_ref

BLOCK_WIDTH = 16  # gs_utils.py:12


def _exp_c(x):
    """Canonical exp: computed in float64, rounded once to float32 (what the fused HIP prep kernel does)."""
    return torch.exp(x.double()).float()


def _viewmat_c(camera_to_world):
    """Canonical viewmat: R = c2w[:3,:3] diag(1,-1,-1), [R^T | -(R^T t)], the 3-term sums left to right."""
    c = camera_to_world.to(torch.float32)
    R = torch.stack([c[:3, 0], -c[:3, 1], -c[:3, 2]], 1)
    t = c[:3, 3]
    vm = torch.zeros(3, 4, dtype=torch.float32)
    vm[:, :3] = R.T
    for r in range(3):
        vm[r, 3] = -((R[0, r] * t[0] + R[1, r] * t[1]) + R[2, r] * t[2])
    return vm


def glue_args(gs_params, camera_to_world, canonical=False):
    """gs_utils.py:31-79: the tensors handed to gsplat (viewmat, scales, quats, opacities, rgbs, viewdirs).

    canonical=False: the reference's own torch ops (bit-exact against the goldens captured from gs_utils.py on
    this CPU; torch's vectorised exp / norm / 3x3 matmul round in implementation-defined ways).
    canonical=True: the same math in the machine-independent arithmetic the fused HIP prep kernel reproduces
    bit for bit -- exp / sigmoid in float64 rounded once, norms as left-to-right sums of rounded squares with
    a correctly rounded sqrt (gsplat_ref.sqrt_rn: torch's CPU float32 sqrt is not correctly rounded), the viewmat's -R^T t as a left-to-right sum; within 1-2 ulp of the torch form
    (tests/test_golden_glue.py)."""
    gs_params = {k: v.float() if v.dtype == torch.half else v for k, v in gs_params.items()}
    if canonical:
        viewmat = _viewmat_c(camera_to_world)
    else:
        R = camera_to_world[:3, :3]
        T = camera_to_world[:3, 3:4]
        R = R @ torch.diag(torch.tensor([1, -1, -1], dtype=R.dtype))         # :35-36
        R_inv = R.T                                                           # :38
        T_inv = -R_inv @ T                                                    # :39
        viewmat = torch.eye(4, dtype=R.dtype)
        viewmat[:3, :3] = R_inv
        viewmat[:3, 3:4] = T_inv
        viewmat = viewmat[:3, :].float()
    means = gs_params["means"]
    q = gs_params["quats"]
    if canonical:
        scales = _exp_c(gs_params["scales"])
        qn = gsplat_ref.sqrt_rn(((q[:, 0] * q[:, 0] + q[:, 1] * q[:, 1]) + q[:, 2] * q[:, 2]) + q[:, 3] * q[:, 3])[:, None]
        quats = q / qn
    else:
        scales = torch.exp(gs_params["scales"])                               # :45
        quats = q / torch.norm(q, dim=-1, keepdim=True)                       # :46
    bad = torch.isnan(quats).any(-1)                                      # :47-51 (only NaNs fail the check)
    quats = quats.clone()
    quats[bad] = torch.tensor([0, 0, 0, 1.0])
    if canonical:
        opacities = (1.0 / (1.0 + torch.exp(-gs_params["opacities"].double()))).float()
    else:
        opacities = torch.sigmoid(gs_params["opacities"])                     # :53-54
    if "features_rest" in gs_params:
        colors = torch.cat([gs_params["features_dc"].unsqueeze(1), gs_params["features_rest"]], dim=1)
    else:
        colors = gs_params["features_dc"].unsqueeze(1)
    n = int(math.sqrt(colors.shape[1]) - 1)
    viewdirs = None
    if n == 0:
        if canonical:
            rgbs = (1.0 / (1.0 + torch.exp(-colors[:, 0, :].double()))).float()
        else:
            rgbs = torch.sigmoid(colors[:, 0, :])                             # :64-65
    else:
        vd = means - camera_to_world[:3, 3]                               # :67
        if canonical:
            nrm = gsplat_ref.sqrt_rn((vd[:, 0] * vd[:, 0] + vd[:, 1] * vd[:, 1]) + vd[:, 2] * vd[:, 2])[:, None]
        else:
            nrm = vd.norm(dim=-1, keepdim=True)
        viewdirs = vd / nrm
        zero = (nrm == 0).squeeze(-1)
        viewdirs[zero] = torch.tensor([0.0, 0.0, 1.0])                    # deterministic stand-in for :72-76
        rgbs = gsplat_ref.spherical_harmonics(n, viewdirs, colors)
        rgbs = torch.clamp(rgbs + 0.5, min=0.0)                           # :79
    return dict(viewmat=viewmat, means=means, scales=scales, quats=quats, opacities=opacities,
                colors=colors, rgbs=rgbs, viewdirs=viewdirs, sh_degree=n)


def rasterize_gaussians_to_singleimg(gs_params, camera_to_world, cx, cy, fx, fy, width, height, background_color,
                                     canonical=True, return_meta=False, **kwargs):
    """gs_utils.py:20-114 with the oracle renderer; canonical=True (default) uses the canonical glue arithmetic
    (the HIP eval path's); return_meta adds the projection and binning outputs for integer comparisons."""
    a = glue_args(gs_params, camera_to_world, canonical=canonical)
    H, W = int(height), int(width)
    xys, depths, radii, conics, comp, tiles, cov3d = gsplat_ref.project_gaussians(
        a["means"], a["scales"], 1, a["quats"], a["viewmat"], float(fx), float(fy), float(cx), float(cy), H, W,
        BLOCK_WIDTH)
    if not return_meta:
        rgb, alpha = gsplat_ref.rasterize_gaussians(xys, depths, radii, conics, tiles, a["rgbs"], a["opacities"], H,
                                                    W, BLOCK_WIDTH, background=background_color, return_alpha=True)
        return torch.clamp(rgb, max=1.0), alpha.unsqueeze(-1)
    # the same steps as gsplat_ref.rasterize_gaussians, keeping the binning for integer comparisons
    meta = dict(xys=xys, depths=depths, radii=radii, conics=conics, num_tiles_hit=tiles, rgbs=a["rgbs"],
                opacities=a["opacities"])
    tx, ty = (W + BLOCK_WIDTH - 1) // BLOCK_WIDTH, (H + BLOCK_WIDTH - 1) // BLOCK_WIDTH
    num_isect = int(tiles.to(torch.int64).sum()) if xys.shape[0] else 0
    if num_isect < 1:
        rgb = torch.ones(H, W, 3) * background_color.float()
        alpha = torch.ones(H, W)  # gsplat v0.1.11 empty-branch quirk: final_T = 0
    else:
        keys, gids, bins = gsplat_ref.bin_and_sort_gaussians(xys, depths, radii, tiles, tx, ty, BLOCK_WIDTH)
        rgb, fT, fidx = gsplat_ref.rasterize_forward(tx, ty, BLOCK_WIDTH, H, W, gids, bins, xys, conics, a["rgbs"],
                                                     a["opacities"], background_color)
        alpha = 1 - fT
        meta.update(isect_sorted=keys, gids_sorted=gids, tile_bins=bins, final_Ts=fT, final_idx=fidx)
    return torch.clamp(rgb, max=1.0), alpha.unsqueeze(-1), meta


def rasterize_gaussians_to_multiimgs(gs_params, cameras):
    rgbs, alphas = [], []
    for c2w in cameras["camera_to_worlds"]:
        rgb, alpha = rasterize_gaussians_to_singleimg(gs_params, c2w, **cameras)
        rgbs.append(rgb)
        alphas.append(alpha)
    return rgbs, alphas
