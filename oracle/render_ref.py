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


def glue_args(gs_params, camera_to_world):
    """gs_utils.py:31-79: the tensors handed to gsplat (viewmat, scales, quats, opacities, rgbs, viewdirs)."""
    gs_params = {k: v.float() if v.dtype == torch.half else v for k, v in gs_params.items()}
    R = camera_to_world[:3, :3]
    T = camera_to_world[:3, 3:4]
    R = R @ torch.diag(torch.tensor([1, -1, -1], dtype=R.dtype))         # :35-36
    R_inv = R.T                                                           # :38
    T_inv = -R_inv @ T                                                    # :39
    viewmat = torch.eye(4, dtype=R.dtype)
    viewmat[:3, :3] = R_inv
    viewmat[:3, 3:4] = T_inv
    means = gs_params["means"]
    scales = torch.exp(gs_params["scales"])                               # :45
    quats = gs_params["quats"] / torch.norm(gs_params["quats"], dim=-1, keepdim=True)  # :46
    bad = torch.isnan(quats).any(-1)                                      # :47-51 (only NaNs fail the check)
    quats = quats.clone()
    quats[bad] = torch.tensor([0, 0, 0, 1.0])
    opacities = torch.sigmoid(gs_params["opacities"])                     # :53-54
    if "features_rest" in gs_params:
        colors = torch.cat([gs_params["features_dc"].unsqueeze(1), gs_params["features_rest"]], dim=1)
    else:
        colors = gs_params["features_dc"].unsqueeze(1)
    n = int(math.sqrt(colors.shape[1]) - 1)
    viewdirs = None
    if n == 0:
        rgbs = torch.sigmoid(colors[:, 0, :])                             # :64-65
    else:
        vd = means - camera_to_world[:3, 3]                               # :67
        nrm = vd.norm(dim=-1, keepdim=True)
        viewdirs = vd / nrm
        zero = (nrm == 0).squeeze(-1)
        viewdirs[zero] = torch.tensor([0.0, 0.0, 1.0])                    # deterministic stand-in for :72-76
        rgbs = gsplat_ref.spherical_harmonics(n, viewdirs, colors)
        rgbs = torch.clamp(rgbs + 0.5, min=0.0)                           # :79
    return dict(viewmat=viewmat[:3, :].float(), means=means, scales=scales, quats=quats, opacities=opacities,
                colors=colors, rgbs=rgbs, viewdirs=viewdirs, sh_degree=n)


def rasterize_gaussians_to_singleimg(gs_params, camera_to_world, cx, cy, fx, fy, width, height, background_color,
                                     **kwargs):
    a = glue_args(gs_params, camera_to_world)
    H, W = int(height), int(width)
    xys, depths, radii, conics, comp, tiles, cov3d = gsplat_ref.project_gaussians(
        a["means"], a["scales"], 1, a["quats"], a["viewmat"], float(fx), float(fy), float(cx), float(cy), H, W,
        BLOCK_WIDTH)
    rgb, alpha = gsplat_ref.rasterize_gaussians(xys, depths, radii, conics, tiles, a["rgbs"], a["opacities"], H, W,
                                                BLOCK_WIDTH, background=background_color, return_alpha=True)
    return torch.clamp(rgb, max=1.0), alpha.unsqueeze(-1)


def rasterize_gaussians_to_multiimgs(gs_params, cameras):
    rgbs, alphas = [], []
    for c2w in cameras["camera_to_worlds"]:
        rgb, alpha = rasterize_gaussians_to_singleimg(gs_params, c2w, **cameras)
        rgbs.append(rgb)
        alphas.append(alpha)
    return rgbs, alphas
