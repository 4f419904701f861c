"""CPU restatement of gsplat v0.1.11 (SH, projection, tile binning, rasterize).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

gsplat is an un-vendored dependency of the reference (pinned
`gsplat.git@v0.1.11`, reference README.md:27); its source is not in
/root/reference.  The algorithm below restates the published v0.1.11 CUDA
kernels (sh.cu `compute_sh_forward_kernel`, forward.cu
`project_gaussians_forward_kernel` / `map_gaussian_to_intersects` /
`get_tile_bin_edges` / `rasterize_forward`, backward.cu
`rasterize_backward_kernel` / `project_gaussians_backward_kernel`, helpers.cuh)
in float32 torch on the CPU.  Reference call sites:
  * utils/gs_utils.py:78      spherical_harmonics(n, viewdirs, colors)
  * utils/gs_utils.py:82-95   project_gaussians(means, scales, 1, quats, viewmat[:3], fx, fy, cx, cy, H, W, 16)
  * utils/gs_utils.py:96-109  rasterize_gaussians(..., background, return_alpha=True)
"""
from __future__ import annotations

import math

import torch

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
SH_C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154,
         -0.4570457994644658, 1.445305721320277, -0.5900435899266435]
SH_C4 = [2.5033429417967046, -1.7701307697799304, 0.9461746957575601, -0.6690465435572892,
         0.10578554691520431, -0.6690465435572892, 0.47308734787878004, -1.7701307697799304,
         0.6258357354491761]

f32 = torch.float32


def sqrt_rn(x: torch.Tensor) -> torch.Tensor:
    """Correctly rounded float32 sqrt (numpy's, i.e. the hardware IEEE instruction).  torch's CPU float32
    sqrt is not correctly rounded (measured: 0.7 % of values off by an ulp on this container's Xeon, 16 % on
    the GPU box's EPYC), which would make the oracle machine-dependent."""
    import numpy as np
    return torch.from_numpy(np.sqrt(x.detach().to(f32).contiguous().numpy()))


def num_sh_bases(degree: int) -> int:
    return (degree + 1) ** 2


def _sh_basis(degree: int, d: torch.Tensor) -> list:
    """Real SH basis (gsplat sh.cu sh_coeffs_to_color), dirs re-normalised."""
    n = d.shape[0]
    b = [torch.full((n,), SH_C0, dtype=f32)]
    if degree < 1:
        return b
    nrm = sqrt_rn(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1] + d[:, 2] * d[:, 2])
    x, y, z = d[:, 0] / nrm, d[:, 1] / nrm, d[:, 2] / nrm
    b += [-SH_C1 * y, SH_C1 * z, -SH_C1 * x]
    if degree < 2:
        return b
    xx, xy, xz, yy, yz, zz = x * x, x * y, x * z, y * y, y * z, z * z
    b += [SH_C2[0] * xy, SH_C2[1] * yz, SH_C2[2] * (2 * zz - xx - yy), SH_C2[3] * xz, SH_C2[4] * (xx - yy)]
    if degree < 3:
        return b
    b += [SH_C3[0] * y * (3 * xx - yy), SH_C3[1] * xy * z, SH_C3[2] * y * (4 * zz - xx - yy),
          SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy), SH_C3[4] * x * (4 * zz - xx - yy), SH_C3[5] * z * (xx - yy),
          SH_C3[6] * x * (xx - 3 * yy)]
    if degree < 4:
        return b
    b += [SH_C4[0] * xy * (xx - yy), SH_C4[1] * yz * (3 * xx - yy), SH_C4[2] * xy * (7 * zz - 1),
          SH_C4[3] * yz * (7 * zz - 3), SH_C4[4] * (zz * (35 * zz - 30) + 3), SH_C4[5] * xz * (7 * zz - 3),
          SH_C4[6] * (xx - yy) * (7 * zz - 1), SH_C4[7] * xz * (xx - 3 * yy),
          SH_C4[8] * (xx * (xx - 3 * yy) - yy * (3 * xx - yy))]
    return b


def spherical_harmonics(degrees_to_use: int, viewdirs: torch.Tensor, coeffs: torch.Tensor) -> torch.Tensor:
    """gsplat.spherical_harmonics forward: colors[N,3] = sum_k basis_k(dir) coeffs[:,k,:]."""
    assert coeffs.shape[-2] >= num_sh_bases(degrees_to_use)
    b = _sh_basis(degrees_to_use, viewdirs.to(f32))
    c = coeffs.to(f32)
    out = b[0][:, None] * c[:, 0, :]
    for k in range(1, len(b)):
        out = out + b[k][:, None] * c[:, k, :]
    return out


def spherical_harmonics_bwd(degrees_to_use: int, viewdirs: torch.Tensor, v_colors: torch.Tensor,
                            num_bases: int) -> torch.Tensor:
    """compute_sh_backward_kernel: v_coeffs[:,k,:] = basis_k * v_colors (0 above degrees_to_use)."""
    b = _sh_basis(degrees_to_use, viewdirs.to(f32))
    out = torch.zeros(v_colors.shape[0], num_bases, 3, dtype=f32)
    for k in range(len(b)):
        out[:, k, :] = b[k][:, None] * v_colors
    return out


def quat_to_rotmat(q: torch.Tensor) -> torch.Tensor:
    """helpers.cuh quat_to_rotmat: q = (w,x,y,z) scaled by s = 1/sqrt(w^2+x^2+y^2+z^2) (gsplat: rsqrtf; the
    canonical form here is the correctly rounded 1/sqrt, sum left to right); returns R[N,3,3] row-major."""
    ss = ((q[:, 0] * q[:, 0] + q[:, 1] * q[:, 1]) + q[:, 2] * q[:, 2]) + q[:, 3] * q[:, 3]
    s = 1.0 / sqrt_rn(ss)
    w, x, y, z = q[:, 0] * s, q[:, 1] * s, q[:, 2] * s, q[:, 3] * s
    R = torch.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
        2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
        2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], -1).reshape(-1, 3, 3)
    return R


def tile_bbox(xy: torch.Tensor, radius: torch.Tensor, tiles_x: int, tiles_y: int, bw: int):
    """helpers.cuh get_tile_bbox/get_bbox: (int) truncation toward zero, clamp to [0, tiles]."""
    tcx, tcy = xy[:, 0] / float(bw), xy[:, 1] / float(bw)
    tr = radius.to(f32) / float(bw)
    x0 = (tcx - tr).to(torch.int32).clamp(min=0).clamp(max=tiles_x)
    x1 = (tcx + tr + 1).to(torch.int32).clamp(min=0).clamp(max=tiles_x)
    y0 = (tcy - tr).to(torch.int32).clamp(min=0).clamp(max=tiles_y)
    y1 = (tcy + tr + 1).to(torch.int32).clamp(min=0).clamp(max=tiles_y)
    return x0, y0, x1, y1


def fov_limits(fx, fy, img_width, img_height):
    """gsplat: tan_fov = 0.5 * img_size / f (double arithmetic, stored as float), lim = 1.3f * tan_fov (float)."""
    import numpy as np
    tan_x = np.float32(0.5 * img_width / float(np.float32(fx)))
    tan_y = np.float32(0.5 * img_height / float(np.float32(fy)))
    return float(np.float32(1.3) * tan_x), float(np.float32(1.3) * tan_y)


def _dot3(a0, a1, a2, b0, b1, b2):
    """Canonical 3-term dot product: (a0 b0 + a1 b1) + a2 b2, every product and sum rounded (no FMA)."""
    return (a0 * b0 + a1 * b1) + a2 * b2


def project_gaussians(means3d, scales, glob_scale, quats, viewmat, fx, fy, cx, cy, img_height, img_width,
                      block_width, clip_thresh=0.01):
    """project_gaussians_forward_kernel.  Returns (xys, depths, radii, conics, comp, num_tiles_hit, cov3d).

    Canonical arithmetic (what the HIP kernel reproduces bit for bit): elementwise fp32 ops in the order
    written, each rounded (no fused multiply-add), sums of products left to right, correctly rounded
    division and sqrt.  gsplat's CUDA build contracts some of these into FMAs (nvcc's default), which moves
    results by an ulp; the canonical form fixes one order so HIP vs oracle can be compared exactly."""
    means3d, scales, quats = means3d.to(f32), scales.to(f32), quats.to(f32)
    vm = viewmat.reshape(-1)[:12].to(f32)
    n = means3d.shape[0]
    px, py, pz = means3d[:, 0], means3d[:, 1], means3d[:, 2]
    tx = vm[0] * px + vm[1] * py + vm[2] * pz + vm[3]
    ty = vm[4] * px + vm[5] * py + vm[6] * pz + vm[7]
    tz = vm[8] * px + vm[9] * py + vm[10] * pz + vm[11]
    keep = tz > clip_thresh
    R = quat_to_rotmat(quats)
    S = glob_scale * scales
    M = R * S[:, None, :]
    # V = M M^T (cov3d), V[r][c] = dot(M[r], M[c])
    V = [[_dot3(M[:, r, 0], M[:, r, 1], M[:, r, 2], M[:, c, 0], M[:, c, 1], M[:, c, 2]) for c in range(3)]
         for r in range(3)]
    cov3d = torch.stack([V[0][0], V[0][1], V[0][2], V[1][1], V[1][2], V[2][2]], -1)
    lim_x, lim_y = fov_limits(fx, fy, img_width, img_height)
    ctx = tz * torch.clamp(tx / tz, min=-lim_x, max=lim_x)
    cty = tz * torch.clamp(ty / tz, min=-lim_y, max=lim_y)
    rz = 1.0 / tz
    rz2 = rz * rz
    # J = [[fx rz, 0, -fx ctx rz2], [0, fy rz, -fy cty rz2]]; T = J W (W = viewmat[:3,:3])
    j00, j02 = fx * rz, -fx * ctx * rz2
    j11, j12 = fy * rz, -fy * cty * rz2
    T0 = [j00 * vm[c] + j02 * vm[8 + c] for c in range(3)]
    T1 = [j11 * vm[4 + c] + j12 * vm[8 + c] for c in range(3)]
    # cov2d = T V T^T
    TV0 = [_dot3(T0[0], T0[1], T0[2], V[0][c], V[1][c], V[2][c]) for c in range(3)]
    TV1 = [_dot3(T1[0], T1[1], T1[2], V[0][c], V[1][c], V[2][c]) for c in range(3)]
    c00 = _dot3(TV0[0], TV0[1], TV0[2], T0[0], T0[1], T0[2])
    c01 = _dot3(TV0[0], TV0[1], TV0[2], T1[0], T1[1], T1[2])
    c11 = _dot3(TV1[0], TV1[1], TV1[2], T1[0], T1[1], T1[2])
    det_orig = c00 * c11 - c01 * c01
    a, b, c = c00 + 0.3, c01, c11 + 0.3
    det = a * c - b * b
    comp = sqrt_rn(torch.clamp(det_orig / det, min=0.0))
    ok = keep & (det != 0)
    inv_det = 1.0 / det
    conics = torch.stack([c * inv_det, -b * inv_det, a * inv_det], -1)
    mid = 0.5 * (a + c)
    disc = sqrt_rn(torch.clamp(mid * mid - det, min=0.1))
    lam1, lam2 = mid + disc, mid - disc
    radius = torch.ceil(3.0 * sqrt_rn(torch.maximum(lam1, lam2)))
    rw = 1.0 / (tz + 1e-6)
    xys = torch.stack([tx * rw * fx + cx, ty * rw * fy + cy], -1)
    tiles_x = (img_width + block_width - 1) // block_width
    tiles_y = (img_height + block_width - 1) // block_width
    x0, y0, x1, y1 = tile_bbox(xys, torch.nan_to_num(radius, nan=0.0, posinf=0.0), tiles_x, tiles_y, block_width)
    area = (x1 - x0) * (y1 - y0)
    vis = ok & (area > 0)
    z2 = lambda t: torch.where(vis.reshape(-1, *([1] * (t.dim() - 1))), t, torch.zeros_like(t))
    out_conics = torch.where(ok[:, None], conics, torch.zeros_like(conics))
    out_cov3d = torch.where(keep[:, None], cov3d, torch.zeros_like(cov3d))
    return (z2(xys), z2(tz), z2(radius).to(torch.int32), out_conics, z2(comp), z2(area).to(torch.int32), out_cov3d)


def map_gaussian_to_intersects(xys, depths, radii, cum_tiles_hit, tiles_x, tiles_y, block_width):
    """map_gaussian_to_intersects: key = tile_id << 32 | int32 bits(depth), val = gaussian id; each Gaussian's
    tiles in row-major order of its bbox, at its cumulative offset."""
    n = xys.shape[0]
    x0, y0, x1, y1 = tile_bbox(xys, radii, tiles_x, tiles_y, block_width)
    num = int(cum_tiles_hit[-1]) if n else 0
    dbits = depths.to(f32).view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    live = radii > 0
    w = torch.where(live, x1 - x0, torch.zeros_like(x1)).to(torch.int64)
    h = torch.where(live, y1 - y0, torch.zeros_like(y1)).to(torch.int64)
    cnt = w * h
    ids = torch.repeat_interleave(torch.arange(n), cnt)
    start = cum_tiles_hit.to(torch.int64) - cnt  # == the exclusive cumsum for every emitting Gaussian
    local = torch.arange(ids.numel(), dtype=torch.int64) - torch.repeat_interleave(
        torch.cumsum(cnt, 0) - cnt, cnt)
    ty = y0.to(torch.int64)[ids] + local // w[ids]
    tx = x0.to(torch.int64)[ids] + local % w[ids]
    pos = start[ids] + local
    keys = torch.zeros(num, dtype=torch.int64)
    gids = torch.zeros(num, dtype=torch.int32)
    keys[pos] = ((ty * tiles_x + tx) << 32) | dbits[ids]
    gids[pos] = ids.to(torch.int32)
    return keys, gids


def bin_and_sort_gaussians(xys, depths, radii, num_tiles_hit, tiles_x, tiles_y, block_width):
    """cumsum -> map_gaussian_to_intersects -> stable sort -> get_tile_bin_edges."""
    cum = torch.cumsum(num_tiles_hit.to(torch.int32), 0, dtype=torch.int32)
    keys, gids = map_gaussian_to_intersects(xys, depths, radii, cum, tiles_x, tiles_y, block_width)
    order = torch.sort(keys, stable=True).indices
    keys_s, gids_s = keys[order], gids[order]
    num_tiles = tiles_x * tiles_y
    bins = torch.zeros(num_tiles, 2, dtype=torch.int32)
    if keys_s.numel():
        tile = (keys_s >> 32).to(torch.int64)
        counts = torch.bincount(tile, minlength=num_tiles)
        ends = torch.cumsum(counts, 0)
        starts = ends - counts
        nz = counts > 0
        bins[nz, 0] = starts[nz].to(torch.int32)
        bins[nz, 1] = ends[nz].to(torch.int32)
    return keys_s, gids_s, bins


def _tile_pixels(tx, ty, bw, H, W):
    ii = torch.arange(bw)
    py = (ty * bw + ii)[:, None].expand(bw, bw).reshape(-1)
    px = (tx * bw + ii)[None, :].expand(bw, bw).reshape(-1)
    inside = (py < H) & (px < W)
    return px, py, inside


def rasterize_forward(tiles_x, tiles_y, bw, H, W, gids_sorted, tile_bins, xys, conics, colors, opacity, background):
    """rasterize_forward: per-pixel front-to-back compositing, vectorised per tile.

    alpha = min(0.999, o*exp(-sigma)); skip sigma<0 or alpha<1/255; stop (without
    adding) once T*(1-alpha) <= 1e-4.  Returns (out_img[H,W,3], final_Ts[H,W],
    final_idx[H,W] int32).
    """
    out = torch.zeros(H, W, 3, dtype=f32)
    final_T = torch.ones(H, W, dtype=f32)
    final_idx = torch.zeros(H, W, dtype=torch.int32)
    bg = background.to(f32)
    op = opacity.reshape(-1).to(f32)
    for ty in range(tiles_y):
        for tx in range(tiles_x):
            t = ty * tiles_x + tx
            r0, r1 = int(tile_bins[t, 0]), int(tile_bins[t, 1])
            px, py, inside = _tile_pixels(tx, ty, bw, H, W)
            pxf, pyf = px.to(f32) + 0.5, py.to(f32) + 0.5
            if r1 > r0:
                g = gids_sorted[r0:r1].long()
                dx = xys[g, 0][None, :] - pxf[:, None]
                dy = xys[g, 1][None, :] - pyf[:, None]
                con = conics[g]
                sigma = 0.5 * (con[:, 0][None] * dx * dx + con[:, 2][None] * dy * dy) + con[:, 1][None] * dx * dy
                alpha = torch.clamp(op[g][None] * torch.exp(-sigma), max=0.999)
                valid = ~((sigma < 0) | (alpha < 1.0 / 255.0))
                a = torch.where(valid, alpha, torch.zeros_like(alpha))
                one_m = 1.0 - a
                Tin = torch.cumprod(torch.cat([torch.ones(one_m.shape[0], 1), one_m[:, :-1]], 1), 1)
                nextT = Tin * one_m
                stop = valid & (nextT <= 1e-4)
                # first stop index per pixel (m if none)
                m = g.numel()
                idxs = torch.arange(m)[None].expand_as(stop)
                first_stop = torch.where(stop, idxs, torch.full_like(idxs, m)).min(1).values
                contrib = valid & (idxs < first_stop[:, None])
                vis = torch.where(contrib, a * Tin, torch.zeros_like(a))
                rgb = vis @ colors[g].to(f32)
                # T after the last contributor
                has_stop = first_stop < m
                lastT = torch.where(has_stop, Tin.gather(1, first_stop.clamp(max=m - 1)[:, None])[:, 0],
                                    Tin[:, -1] * one_m[:, -1])
                last_c = torch.where(contrib, idxs, torch.full_like(idxs, -1)).max(1).values
                fidx = torch.where(last_c >= 0, last_c + r0, torch.zeros_like(last_c)).to(torch.int32)
            else:
                rgb = torch.zeros(px.numel(), 3, dtype=f32)
                lastT = torch.ones(px.numel(), dtype=f32)
                fidx = torch.zeros(px.numel(), dtype=torch.int32)
            sel = inside
            out[py[sel], px[sel]] = rgb[sel] + lastT[sel][:, None] * bg[None]
            final_T[py[sel], px[sel]] = lastT[sel]
            final_idx[py[sel], px[sel]] = fidx[sel]
    return out, final_T, final_idx


def rasterize_gaussians(xys, depths, radii, conics, num_tiles_hit, colors, opacity, img_height, img_width,
                        block_width, background=None, return_alpha=False):
    """gsplat.rasterize_gaussians (3-channel path) forward."""
    colors = colors.to(f32)
    if background is None:
        background = torch.ones(colors.shape[-1], dtype=f32)
    tiles_x = (img_width + block_width - 1) // block_width
    tiles_y = (img_height + block_width - 1) // block_width
    num_isect = int(num_tiles_hit.to(torch.int64).sum()) if xys.shape[0] else 0
    if num_isect < 1:
        out = torch.ones(img_height, img_width, colors.shape[-1], dtype=f32) * background
        final_T = torch.zeros(img_height, img_width, dtype=f32)  # gsplat v0.1.11 empty-branch quirk
        return (out, 1 - final_T) if return_alpha else out
    _, gids, bins = bin_and_sort_gaussians(xys, depths, radii, num_tiles_hit, tiles_x, tiles_y, block_width)
    out, final_T, _ = rasterize_forward(tiles_x, tiles_y, block_width, img_height, img_width, gids, bins, xys,
                                        conics, colors, opacity, background)
    return (out, 1 - final_T) if return_alpha else out


def rasterize_backward(tiles_x, tiles_y, bw, H, W, gids_sorted, tile_bins, xys, conics, colors, opacity,
                       background, final_Ts, final_idx, v_out, v_out_alpha):
    """rasterize_backward_kernel: back-to-front replay from final_idx (alpha clamp 0.99).

    Returns (v_xy[N,2], v_conic[N,3], v_rgb[N,3], v_opacity[N,1])."""
    n = xys.shape[0]
    v_xy = torch.zeros(n, 2, dtype=f32)
    v_conic = torch.zeros(n, 3, dtype=f32)
    v_rgb = torch.zeros(n, 3, dtype=f32)
    v_op = torch.zeros(n, dtype=f32)
    op = opacity.reshape(-1).to(f32)
    bg = background.to(f32)
    for ty in range(tiles_y):
        for tx in range(tiles_x):
            t = ty * tiles_x + tx
            r0, r1 = int(tile_bins[t, 0]), int(tile_bins[t, 1])
            if r1 <= r0:
                continue
            px, py, inside = _tile_pixels(tx, ty, bw, H, W)
            if not bool(inside.any()):
                continue
            px, py = px[inside], py[inside]
            pxf, pyf = px.to(f32) + 0.5, py.to(f32) + 0.5
            Tf = final_Ts[py, px]
            bfin = final_idx[py, px].long()
            vo = v_out[py, px]
            voa = v_out_alpha[py, px]
            g = gids_sorted[r0:r1].long()
            m = g.numel()
            pos = torch.arange(r0, r1)[None]
            dx = xys[g, 0][None] - pxf[:, None]
            dy = xys[g, 1][None] - pyf[:, None]
            con = conics[g]
            sigma = 0.5 * (con[:, 0][None] * dx * dx + con[:, 2][None] * dy * dy) + con[:, 1][None] * dx * dy
            vis = torch.exp(-sigma)
            alpha = torch.clamp(op[g][None] * vis, max=0.99)
            valid = (pos <= bfin[:, None]) & ~((sigma < 0) | (alpha < 1.0 / 255.0))
            a = torch.where(valid, alpha, torch.zeros_like(alpha))
            ra = 1.0 / (1.0 - a)
            # back-to-front: T_j = T_final * prod_{k>=j} ra_k (sequential, reversed)
            Tj = Tf[:, None] * torch.flip(torch.cumprod(torch.flip(ra, [1]), 1), [1])
            fac = a * Tj
            c = colors[g].to(f32)  # [m,3]
            contrib = fac[:, :, None] * c[None]  # [P,m,3]
            # buffer_j = sum_{k>j} contrib_k  (accumulated back to front)
            rc = torch.flip(torch.cumsum(torch.flip(contrib, [1]), 1), [1])
            buf = rc - contrib
            v_alpha = ((c[None] * Tj[:, :, None] - buf * ra[:, :, None]) * vo[:, None, :]).sum(-1)
            v_alpha = v_alpha + Tf[:, None] * ra * voa[:, None]
            v_alpha = v_alpha - (Tf[:, None] * ra)[:, :, None].mul(bg[None, None] * vo[:, None, :]).sum(-1)
            v_sigma = -op[g][None] * vis * v_alpha
            w = valid.to(f32)
            g_rgb = (fac[:, :, None] * vo[:, None, :] * w[:, :, None]).sum(0)
            g_con = torch.stack([0.5 * v_sigma * dx * dx, v_sigma * dx * dy, 0.5 * v_sigma * dy * dy], -1)
            g_con = (g_con * w[:, :, None]).sum(0)
            g_xy = torch.stack([v_sigma * (con[:, 0][None] * dx + con[:, 1][None] * dy),
                                v_sigma * (con[:, 1][None] * dx + con[:, 2][None] * dy)], -1)
            g_xy = (g_xy * w[:, :, None]).sum(0)
            g_o = (vis * v_alpha * w).sum(0)
            v_rgb.index_add_(0, g, g_rgb)
            v_conic.index_add_(0, g, g_con)
            v_xy.index_add_(0, g, g_xy)
            v_op.index_add_(0, g, g_o)
    return v_xy, v_conic, v_rgb, v_op[:, None]


def project_gaussians_backward(means3d, scales, glob_scale, quats, viewmat, fx, fy, cov3d, radii, conics,
                               compensation, v_xy, v_depth, v_conic, v_comp):
    """project_gaussians_backward_kernel (no frustum clamp in the EWA vjp; quat grad w.r.t. normalised q).

    Returns (v_mean3d[N,3], v_scale[N,3], v_quat[N,4])."""
    vm = viewmat.reshape(-1)[:12].to(f32)
    W = vm.reshape(3, 4)[:, :3]
    p = means3d.to(f32)
    tx = vm[0] * p[:, 0] + vm[1] * p[:, 1] + vm[2] * p[:, 2] + vm[3]
    ty = vm[4] * p[:, 0] + vm[5] * p[:, 1] + vm[6] * p[:, 2] + vm[7]
    tz = vm[8] * p[:, 0] + vm[9] * p[:, 1] + vm[10] * p[:, 2] + vm[11]
    rw = 1.0 / (tz + 1e-6)
    vpx, vpy = fx * v_xy[:, 0], fy * v_xy[:, 1]
    vview = torch.stack([vpx * rw, vpy * rw, -(vpx * tx + vpy * ty) * rw * rw], -1)
    v_mean = vview @ W  # transform_4x3_rot_only_transposed
    v_mean = v_mean + v_depth[:, None] * W[2][None]
    X0, X1, X2 = conics[:, 0], conics[:, 1], conics[:, 2]
    X = torch.stack([X0, X1, X1, X2], -1).reshape(-1, 2, 2)
    G = torch.stack([v_conic[:, 0], 0.5 * v_conic[:, 1], 0.5 * v_conic[:, 1], v_conic[:, 2]], -1).reshape(-1, 2, 2)
    vS = -(X @ G @ X)
    vc2 = torch.stack([vS[:, 0, 0], vS[:, 1, 0] + vS[:, 0, 1], vS[:, 1, 1]], -1)
    inv_det = X0 * X2 - X1 * X1
    one_m = 1.0 - compensation * compensation
    vsq = v_comp * 0.5 / (compensation + 1e-6)
    vc2 = vc2 + torch.stack([vsq * (one_m * X0 - 0.3 * inv_det), 2 * vsq * (one_m * X1),
                             vsq * (one_m * X2 - 0.3 * inv_det)], -1)
    c = cov3d
    V = torch.stack([c[:, 0], c[:, 1], c[:, 2], c[:, 1], c[:, 3], c[:, 4], c[:, 2], c[:, 4], c[:, 5]], -1).reshape(-1, 3, 3)
    rz = 1.0 / tz
    rz2, rz3 = rz * rz, rz * rz * rz
    n = p.shape[0]
    J = torch.zeros(n, 3, 3, dtype=f32)
    J[:, 0, 0] = fx * rz
    J[:, 0, 2] = -fx * tx * rz2
    J[:, 1, 1] = fy * rz
    J[:, 1, 2] = -fy * ty * rz2
    T = J @ W
    Gc = torch.zeros(n, 3, 3, dtype=f32)
    Gc[:, 0, 0] = vc2[:, 0]
    Gc[:, 0, 1] = 0.5 * vc2[:, 1]
    Gc[:, 1, 0] = 0.5 * vc2[:, 1]
    Gc[:, 1, 1] = vc2[:, 2]
    vV = T.transpose(1, 2) @ Gc @ T
    vT = Gc @ T @ V.transpose(1, 2) + Gc.transpose(1, 2) @ T @ V
    vc3 = torch.stack([vV[:, 0, 0], vV[:, 0, 1] + vV[:, 1, 0], vV[:, 0, 2] + vV[:, 2, 0], vV[:, 1, 1],
                       vV[:, 1, 2] + vV[:, 2, 1], vV[:, 2, 2]], -1)
    vJ = vT @ W.T
    vt = torch.stack([-fx * rz2 * vJ[:, 0, 2], -fy * rz2 * vJ[:, 1, 2],
                      -fx * rz2 * vJ[:, 0, 0] + 2 * fx * tx * rz3 * vJ[:, 0, 2] - fy * rz2 * vJ[:, 1, 1]
                      + 2 * fy * ty * rz3 * vJ[:, 1, 2]], -1)
    v_mean = v_mean + vt @ W
    # scale / rotation
    q = quats.to(f32)
    R = quat_to_rotmat(q)
    s = glob_scale * scales.to(f32)
    vVs = torch.stack([vc3[:, 0], 0.5 * vc3[:, 1], 0.5 * vc3[:, 2], 0.5 * vc3[:, 1], vc3[:, 3], 0.5 * vc3[:, 4],
                       0.5 * vc3[:, 2], 0.5 * vc3[:, 4], vc3[:, 5]], -1).reshape(-1, 3, 3)
    M = R * s[:, None, :]
    vM = 2.0 * vVs @ M
    v_scale = (R * vM).sum(1) * glob_scale
    vR = vM * s[:, None, :]
    sn = torch.rsqrt((q * q).sum(-1))
    w, x, y, z = q[:, 0] * sn, q[:, 1] * sn, q[:, 2] * sn, q[:, 3] * sn
    VR = lambda col, row: vR[:, row, col]
    v_quat = torch.stack([
        2 * (x * (VR(1, 2) - VR(2, 1)) + y * (VR(2, 0) - VR(0, 2)) + z * (VR(0, 1) - VR(1, 0))),
        2 * (-2 * x * (VR(1, 1) + VR(2, 2)) + y * (VR(0, 1) + VR(1, 0)) + z * (VR(0, 2) + VR(2, 0))
             + w * (VR(1, 2) - VR(2, 1))),
        2 * (x * (VR(0, 1) + VR(1, 0)) - 2 * y * (VR(0, 0) + VR(2, 2)) + z * (VR(1, 2) + VR(2, 1))
             + w * (VR(2, 0) - VR(0, 2))),
        2 * (x * (VR(0, 2) + VR(2, 0)) + y * (VR(1, 2) + VR(2, 1)) - 2 * z * (VR(0, 0) + VR(1, 1))
             + w * (VR(0, 1) - VR(1, 0))),
    ], -1)
    live = (radii > 0)[:, None]
    zero = lambda t: torch.where(live, t, torch.zeros_like(t))
    return zero(v_mean), zero(v_scale), zero(v_quat)


def psnr_u8(pred: torch.Tensor, gt: torch.Tensor) -> torch.Tensor:
    """train.py:104-113 (x*255).to(uint8) then utils/metrics.py:26-29, :89-91 psnr on /255."""
    p = (pred * 255).to(torch.uint8)
    g = (gt * 255).to(torch.uint8)
    # metrics.py:26-29: a batch is divided by 255 only when its max exceeds 1
    p = p / 255.0 if p.max() > 1 else p.to(f32)
    g = g / 255.0 if g.max() > 1 else g.to(f32)
    mse = ((p - g) ** 2).reshape(p.shape[0], -1).mean(1, keepdim=True)
    return 20 * torch.log10(1.0 / torch.sqrt(mse))


_ = math  # keep import for callers computing FOVs
