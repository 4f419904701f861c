"""Deterministic synthetic Gaussian scenes and cameras.

The reference's datasets (Objaverse/GSO OOD test sets, reference
README.md:31-59) are Google-Drive downloads that are unavailable offline, so
the harness builds scenes of the same shape: N Gaussians with the nerfstudio
attribute layout (`means`, `scales` (log), `quats` (w,x,y,z, unnormalised),
`opacities` (logit), `features_dc`, `features_rest` [N,(d+1)^2-1,3]),
already normalised as `MinMaxScaler.fit_transform` does
(reference utils/transform_utils.py:64-91: ratio-preserving, centred in
[0,1]^3), plus the 9 OOD test cameras (elevation 70/80/90 x azimuth
0/120/240, reference dataset/GS.py:223-238).
"""
from __future__ import annotations

import math
from typing import Dict

import torch

BLENDER_FOV = 0.6911112070083618  # 50 mm lens on a 36 mm sensor


def minmax_normalize(x: torch.Tensor) -> torch.Tensor:
    """MinMaxScaler(feature_range=(0,1), preserve_ratio=True).fit_transform (transform_utils.py:64-91)."""
    dmin = x.min(0).values
    dmax = x.max(0).values
    scale = torch.min(1.0 / (dmax - dmin))
    sx = x * scale
    mid = (sx.min(0).values + sx.max(0).values) / 2
    return sx + (0.5 - mid)


def make_scene(n: int, sh_degree: int = 1, seed: int = 0, unique_voxels: bool = False,
               grid_resolution: int = 384) -> Dict[str, torch.Tensor]:
    """CPU float32 scene of `n` Gaussians (seeded).  `unique_voxels` drops points that share a
    stage-0 voxel at `grid_resolution` (used by parity fixtures, SURVEY.md §7 hard part 2)."""
    g = torch.Generator().manual_seed(seed)
    n_surf = int(round(n * 0.95))
    # union of 4 random ellipsoids, surface samples
    centers = torch.rand(4, 3, generator=g) * 0.6 - 0.3
    radii = torch.rand(4, 3, generator=g) * 0.35 + 0.15
    which = torch.randint(0, 4, (n_surf,), generator=g)
    d = torch.randn(n_surf, 3, generator=g)
    d = d / d.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    surf = centers[which] + d * radii[which]
    vol = torch.rand(n - n_surf, 3, generator=g) * 1.2 - 0.6
    means = minmax_normalize(torch.cat([surf, vol], 0))
    perm = torch.randperm(n, generator=g)
    means = means[perm].contiguous()
    if unique_voxels:
        vox = torch.floor(means * grid_resolution).long()
        key = (vox[:, 0] * (grid_resolution + 1) + vox[:, 1]) * (grid_resolution + 1) + vox[:, 2]
        first = torch.full((int(key.max()) + 1,), n, dtype=torch.long)
        first.scatter_reduce_(0, key, torch.arange(n), reduce="amin")
        keep = first[key] == torch.arange(n)
        means = means[keep].contiguous()
    m = means.shape[0]
    scales = math.log(0.004) + 0.5 * torch.randn(m, 3, generator=g)
    quats = torch.randn(m, 4, generator=g)
    opac = 1.0 + 1.5 * torch.randn(m, 1, generator=g)
    dc = 0.6 * torch.randn(m, 3, generator=g)
    scene = {"means": means, "scales": scales, "quats": quats, "opacities": opac, "features_dc": dc}
    nrest = (sh_degree + 1) ** 2 - 1
    if nrest > 0:
        scene["features_rest"] = 0.1 * torch.randn(m, nrest, 3, generator=g)
    return {k: v.float().contiguous() for k, v in scene.items()}


def look_at_c2w(eye: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """OpenGL/Blender camera_to_world (x right, y up, looking down -z), as nerfstudio stores it."""
    f = target - eye
    f = f / f.norm()
    up = torch.tensor([0.0, 0.0, 1.0], dtype=torch.float64)
    r = torch.linalg.cross(f, up)
    if r.norm() < 1e-6:
        r = torch.linalg.cross(f, torch.tensor([0.0, 1.0, 0.0], dtype=torch.float64))
    r = r / r.norm()
    u = torch.linalg.cross(r, f)
    c2w = torch.eye(4, dtype=torch.float64)
    c2w[:3, 0], c2w[:3, 1], c2w[:3, 2], c2w[:3, 3] = r, u, -f, eye
    return c2w


def make_cameras(width: int, height: int, n_views: int = 9, radius: float = 2.0, fov: float = BLENDER_FOV,
                 center=(0.5, 0.5, 0.5)) -> Dict:
    """OOD test cameras: elevations 70/80/90 deg x azimuths 0/120/240 (first `n_views`)."""
    tgt = torch.tensor(center, dtype=torch.float64)
    c2ws = []
    for elev in (70.0, 80.0, 90.0):
        for az in (0.0, 120.0, 240.0):
            e, a = math.radians(elev), math.radians(az)
            eye = tgt + radius * torch.tensor([math.cos(e) * math.cos(a), math.cos(e) * math.sin(a), math.sin(e)],
                                              dtype=torch.float64)
            c2ws.append(look_at_c2w(eye, tgt))
    c2ws = c2ws[:n_views]
    while len(c2ws) < n_views:  # extra views on a ring at 45 deg
        k = len(c2ws)
        e, a = math.radians(45.0), math.radians(37.0 * k)
        eye = tgt + radius * torch.tensor([math.cos(e) * math.cos(a), math.cos(e) * math.sin(a), math.sin(e)],
                                          dtype=torch.float64)
        c2ws.append(look_at_c2w(eye, tgt))
    focal = width / (2.0 * math.tan(fov / 2.0))
    return {
        "camera_to_worlds": torch.stack(c2ws).float(),
        "fx": float(focal), "fy": float(focal), "cx": width / 2.0, "cy": height / 2.0,
        "width": int(width), "height": int(height),
        "background_color": torch.zeros(3, dtype=torch.float32),
    }


def to_device(d, device):
    if isinstance(d, dict):
        return {k: to_device(v, device) for k, v in d.items()}
    if isinstance(d, torch.Tensor):
        return d.to(device)
    return d
