"""Drop-in replacement for the gsplat v0.1.11 Python API used by SplatFormer.

Same names, argument order, return tuples and autograd behaviour as
`gsplat.spherical_harmonics`, `gsplat.project_gaussians` and
`gsplat.rasterize_gaussians` as called from reference utils/gs_utils.py:78,
:82-95 and :96-109.  Every op runs on the libsfx HIP kernels
(csrc/render.hip, csrc/sort.hip); there is no CPU path.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
from torch import Tensor

from . import _lib
from ._lib import call, ptr, stream

__all__ = ["spherical_harmonics", "project_gaussians", "rasterize_gaussians", "num_sh_bases", "deg_from_sh",
           "bin_and_sort_gaussians", "compute_cumulative_intersects"]


def num_sh_bases(degree: int) -> int:
    return (degree + 1) ** 2


def deg_from_sh(num_bases: int) -> int:
    d = {1: 0, 4: 1, 9: 2, 16: 3, 25: 4}
    if num_bases not in d:
        raise ValueError(f"invalid number of SH bases: {num_bases}")
    return d[num_bases]


# exact contribution culling (ABI v9, csrc/render.hip): the rasterizer runs over the (Gaussian, tile) pairs that
# can reach alpha >= 1/255 -- forward outputs bit-identical, gradients the same sums in another atomic order.
# SFX_RENDER_CULL=0 restores gsplat's full 3-sigma lists.
CULL = os.environ.get("SFX_RENDER_CULL", "1") != "0"
_I, _P = _lib.I, _lib.P
_lib.register("sfx_isect_count_cull_views", [_I, _I, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P])
_lib.register("sfx_isect_emit_cull_views", [_I, _I, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _lib.L, _P])
_lib.register("sfx_pack_raster_records", [_I, _P, _P, _P, _P, _P, _P])
_lib.register("sfx_rasterize_fwd_views_quad", [_I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P])
_lib.register("sfx_rasterize_bwd_quad", [_I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                         _P, _P, _P])


def _f32(t: Tensor) -> Tensor:
    return t.contiguous() if t.dtype == torch.float32 else t.float().contiguous()


# ---------------------------------------------------------------------------
class _SphericalHarmonics(torch.autograd.Function):
    @staticmethod
    def forward(ctx, degrees_to_use: int, viewdirs: Tensor, coeffs: Tensor):
        _lib.require_gpu(coeffs)
        n, nb = coeffs.shape[0], coeffs.shape[-2]
        viewdirs, coeffs = _f32(viewdirs), _f32(coeffs)
        colors = torch.empty(n, 3, device=coeffs.device, dtype=torch.float32)
        call("sfx_sh_fwd", n, nb, degrees_to_use, ptr(viewdirs), ptr(coeffs), ptr(colors), stream())
        ctx.degrees_to_use = degrees_to_use
        ctx.num_bases = nb
        ctx.save_for_backward(viewdirs)
        return colors

    @staticmethod
    def backward(ctx, v_colors: Tensor):
        (viewdirs,) = ctx.saved_tensors
        n = viewdirs.shape[0]
        v_colors = _f32(v_colors)
        v_coeffs = torch.empty(n, ctx.num_bases, 3, device=v_colors.device, dtype=torch.float32)
        call("sfx_sh_bwd", n, ctx.num_bases, ctx.degrees_to_use, ptr(viewdirs), ptr(v_colors), ptr(v_coeffs), stream())
        return None, None, v_coeffs


def spherical_harmonics(degrees_to_use: int, viewdirs: Tensor, coeffs: Tensor) -> Tensor:
    """Colors [N,3] from SH coeffs [N,K,3] along viewdirs [N,3] (gsplat v0.1.11 semantics)."""
    assert coeffs.shape[-2] >= num_sh_bases(degrees_to_use)
    return _SphericalHarmonics.apply(degrees_to_use, viewdirs.contiguous(), coeffs.contiguous())


# ---------------------------------------------------------------------------
class _ProjectGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3d, scales, glob_scale, quats, viewmat, fx, fy, cx, cy, img_height, img_width,
                block_width, clip_thresh=0.01):
        _lib.require_gpu(means3d)
        n = means3d.shape[0]
        dev = means3d.device
        means3d, scales, quats = _f32(means3d), _f32(scales), _f32(quats)
        vm = _f32(viewmat.reshape(-1)[:12])
        xys = torch.empty(n, 2, device=dev, dtype=torch.float32)
        depths = torch.empty(n, device=dev, dtype=torch.float32)
        radii = torch.empty(n, device=dev, dtype=torch.int32)
        conics = torch.empty(n, 3, device=dev, dtype=torch.float32)
        comp = torch.empty(n, device=dev, dtype=torch.float32)
        tiles = torch.empty(n, device=dev, dtype=torch.int32)
        cov3d = torch.empty(n, 6, device=dev, dtype=torch.float32)
        call("sfx_project_fwd", n, ptr(means3d), ptr(scales), float(glob_scale), ptr(quats), ptr(vm), float(fx),
             float(fy), float(cx), float(cy), int(img_height), int(img_width), int(block_width), float(clip_thresh),
             ptr(xys), ptr(depths), ptr(radii), ptr(conics), ptr(comp), ptr(tiles), ptr(cov3d), stream())
        ctx.glob_scale, ctx.fx, ctx.fy = float(glob_scale), float(fx), float(fy)
        ctx.save_for_backward(means3d, scales, quats, vm, cov3d, radii, conics, comp)
        ctx.mark_non_differentiable(radii, tiles)
        return xys, depths, radii, conics, comp, tiles, cov3d

    @staticmethod
    def backward(ctx, v_xys, v_depths, v_radii, v_conics, v_comp, v_tiles, v_cov3d):
        means3d, scales, quats, vm, cov3d, radii, conics, comp = ctx.saved_tensors
        n = means3d.shape[0]
        dev = means3d.device
        z = lambda g, *shape: _f32(g) if g is not None else torch.zeros(*shape, device=dev, dtype=torch.float32)
        v_xys, v_depths = z(v_xys, n, 2), z(v_depths, n)
        v_conics, v_comp = z(v_conics, n, 3), z(v_comp, n)
        v_mean = torch.empty(n, 3, device=dev, dtype=torch.float32)
        v_scale = torch.empty(n, 3, device=dev, dtype=torch.float32)
        v_quat = torch.empty(n, 4, device=dev, dtype=torch.float32)
        call("sfx_project_bwd", n, ptr(means3d), ptr(scales), ctx.glob_scale, ptr(quats), ptr(vm), ctx.fx, ctx.fy,
             ptr(cov3d), ptr(radii), ptr(conics), ptr(comp), ptr(v_xys), ptr(v_depths), ptr(v_conics), ptr(v_comp),
             ptr(v_mean), ptr(v_scale), ptr(v_quat), None, None, stream())
        return (v_mean, v_scale, None, v_quat) + (None,) * 9


def project_gaussians(means3d: Tensor, scales: Tensor, glob_scale: float, quats: Tensor, viewmat: Tensor,
                      fx: float, fy: float, cx: float, cy: float, img_height: int, img_width: int,
                      block_width: int, clip_thresh: float = 0.01) -> Tuple[Tensor, ...]:
    """(xys, depths, radii, conics, compensation, num_tiles_hit, cov3d) -- gsplat v0.1.11 contract."""
    assert block_width > 1 and block_width <= 16, "block_width must be between 2 and 16"
    return _ProjectGaussians.apply(means3d.contiguous(), scales.contiguous(), glob_scale, quats.contiguous(),
                                   viewmat.contiguous(), fx, fy, cx, cy, img_height, img_width, block_width,
                                   clip_thresh)


# ---------------------------------------------------------------------------
def compute_cumulative_intersects(num_tiles_hit: Tensor) -> Tuple[int, Tensor]:
    """Device int32 inclusive scan; returns (num_intersects, cum_tiles_hit).  One host sync (as gsplat)."""
    n = num_tiles_hit.shape[0]
    dev = num_tiles_hit.device
    nth = num_tiles_hit.to(torch.int32).contiguous()
    cum = torch.empty(n, device=dev, dtype=torch.int32)
    total = torch.empty(1, device=dev, dtype=torch.int32)
    ws = _lib.workspace(_lib.fn("sfx_scan_workspace_bytes")(n), dev)
    call("sfx_scan_i32", n, ptr(nth), ptr(cum), 1, ptr(ws), ws.numel(), ptr(total), stream())
    return int(total.item()), cum


def bin_and_sort_gaussians(num_points: int, num_intersects: int, xys: Tensor, depths: Tensor, radii: Tensor,
                           cum_tiles_hit: Tensor, tile_bounds, block_width: int):
    """map_gaussian_to_intersects -> stable radix sort -> tile bin edges (all on device)."""
    dev = xys.device
    tiles_x, tiles_y = int(tile_bounds[0]), int(tile_bounds[1])
    num_tiles = tiles_x * tiles_y
    isect_ids = torch.empty(num_intersects, device=dev, dtype=torch.int64)
    gids = torch.empty(num_intersects, device=dev, dtype=torch.int32)
    call("sfx_isect_emit", num_points, ptr(xys), ptr(depths), ptr(radii), ptr(cum_tiles_hit), tiles_x, tiles_y,
         block_width, ptr(isect_ids), ptr(gids), stream())
    isect_sorted = torch.empty_like(isect_ids)
    gids_sorted = torch.empty_like(gids)
    tile_bits = max(1, int(num_tiles - 1).bit_length())
    ws = _lib.workspace(_lib.fn("sfx_sort_workspace_bytes")(num_intersects), dev)
    call("sfx_sort_pairs_u64", num_intersects, ptr(isect_ids), ptr(gids), ptr(isect_sorted), ptr(gids_sorted), 0,
         32 + tile_bits, ptr(ws), ws.numel(), stream())
    tile_bins = torch.empty(num_tiles, 2, device=dev, dtype=torch.int32)
    call("sfx_tile_bins", num_intersects, ptr(isect_sorted), num_tiles, ptr(tile_bins), stream())
    return isect_ids, gids, isect_sorted, gids_sorted, tile_bins


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xys, depths, radii, conics, num_tiles_hit, colors, opacity, img_height, img_width,
                block_width, background, return_alpha):
        _lib.require_gpu(xys)
        dev = xys.device
        n = xys.shape[0]
        H, W, bw = int(img_height), int(img_width), int(block_width)
        tiles_x, tiles_y = (W + bw - 1) // bw, (H + bw - 1) // bw
        xys, conics, colors, opacity, background = map(_f32, (xys, conics, colors, opacity, background))
        culled = CULL and bw == 16 and n > 0
        if culled:
            # gsplat's own list only decides the empty-image branch: one device flag, read back together with the
            # culled list's total (one host sync per view, as gsplat's num_intersects read)
            num_isect, kept_total, kept_cum = _culled_counts(n, num_tiles_hit, xys, radii.to(torch.int32).contiguous(),
                                                             conics, opacity, H, W, tiles_x, tiles_y)
        else:
            num_isect, cum = compute_cumulative_intersects(num_tiles_hit) if n else (0, None)
        ctx.num_isect = num_isect
        if num_isect < 1:
            out = torch.ones(H, W, colors.shape[-1], device=dev) * background
            gids_sorted = torch.zeros(0, device=dev, dtype=torch.int32)
            tile_bins = torch.zeros(0, 2, device=dev, dtype=torch.int32)
            final_Ts = torch.zeros(H, W, device=dev)  # gsplat v0.1.11 empty-branch quirk (alpha == 1)
            final_idx = torch.zeros(H, W, device=dev, dtype=torch.int32)
            alpha = 1 - final_Ts
        elif culled:
            out, alpha, final_Ts, final_idx, gids_sorted, tile_bins = _culled_forward(
                n, xys, _f32(depths), radii.to(torch.int32).contiguous(), conics, colors, opacity, background, H, W,
                tiles_x, tiles_y, kept_total, kept_cum)
            ctx.quad = True
        else:
            _, _, _, gids_sorted, tile_bins = bin_and_sort_gaussians(
                n, num_isect, _f32(xys), _f32(depths), radii.to(torch.int32).contiguous(), cum,
                (tiles_x, tiles_y, 1), bw)
            out = torch.empty(H, W, 3, device=dev, dtype=torch.float32)
            final_Ts = torch.empty(H, W, device=dev, dtype=torch.float32)
            final_idx = torch.empty(H, W, device=dev, dtype=torch.int32)
            alpha = torch.empty(H, W, device=dev, dtype=torch.float32)
            call("sfx_rasterize_fwd", tiles_x, tiles_y, bw, H, W, ptr(gids_sorted), ptr(tile_bins), ptr(xys),
                 ptr(conics), ptr(colors), ptr(opacity), ptr(background), ptr(final_Ts), ptr(final_idx), ptr(out),
                 ptr(alpha), stream())
        ctx.quad = getattr(ctx, "quad", False)
        ctx.img = (H, W, bw, tiles_x, tiles_y)
        ctx.save_for_backward(gids_sorted, tile_bins, xys, conics, colors, opacity, background, final_Ts, final_idx)
        if return_alpha:
            return out, alpha
        return out

    @staticmethod
    def backward(ctx, v_out_img, v_out_alpha=None):
        gids_sorted, tile_bins, xys, conics, colors, opacity, background, final_Ts, final_idx = ctx.saved_tensors
        H, W, bw, tiles_x, tiles_y = ctx.img
        dev = xys.device
        n = xys.shape[0]
        v_xy = torch.zeros(n, 2, device=dev)
        v_conic = torch.zeros(n, 3, device=dev)
        v_rgb = torch.zeros(n, 3, device=dev)
        v_op = torch.zeros_like(opacity)
        if ctx.num_isect >= 1:
            v_out_img = _f32(v_out_img)
            v_out_alpha = _f32(v_out_alpha) if v_out_alpha is not None else None
            v_xy_abs = torch.zeros(n, 2, device=dev)
            call("sfx_rasterize_bwd_quad" if ctx.quad else "sfx_rasterize_bwd", tiles_x, tiles_y, bw, H, W,
                 ptr(gids_sorted), ptr(tile_bins), ptr(xys),
                 ptr(conics), ptr(colors), ptr(opacity), ptr(background), ptr(final_Ts), ptr(final_idx),
                 ptr(v_out_img), ptr(v_out_alpha), ptr(v_xy), ptr(v_xy_abs), ptr(v_conic), ptr(v_rgb), ptr(v_op),
                 stream())
            xys.absgrad = v_xy_abs
        return (v_xy, None, None, v_conic, None, v_rgb, v_op) + (None,) * 5


def _culled_counts(n, num_tiles_hit, xys, radii, conics, opacity, H, W, tiles_x, tiles_y):
    """-> (1 if gsplat's 3-sigma list is non-empty else 0, culled list length, its inclusive scan): the surviving
    tile counts and their scan on device, then ONE host read of [max(num_tiles_hit) > 0, culled total]."""
    dev = xys.device
    kept = torch.empty(n, device=dev, dtype=torch.int32)
    call("sfx_isect_count_cull_views", n, n, ptr(xys), ptr(conics), ptr(opacity), ptr(radii), tiles_x, tiles_y, 16, H,
         W, ptr(kept), stream())
    cum = torch.empty(n, device=dev, dtype=torch.int32)
    flags = torch.empty(2, device=dev, dtype=torch.int32)  # [gsplat non-empty, culled total]
    ws = _lib.workspace(_lib.fn("sfx_scan_workspace_bytes")(n), dev)
    call("sfx_scan_i32", n, ptr(kept), ptr(cum), 1, ptr(ws), ws.numel(), ptr(flags[1:]), stream())
    flags[0] = (num_tiles_hit.max() > 0).to(torch.int32)
    nonempty, total = flags.tolist()
    return nonempty, total, cum


def _culled_forward(n, xys, depths, radii, conics, colors, opacity, background, H, W, tiles_x, tiles_y, total, cum):
    """The forward over the culled list (single view): culled emission over the surviving tile counts' scan (from
    _culled_counts) -> the same stable sort and bins -> rasterize_fwd_views_quad.  Called when gsplat's own list is
    non-empty."""
    dev = xys.device
    num_tiles = tiles_x * tiles_y
    final_Ts = torch.empty(H, W, device=dev, dtype=torch.float32)
    final_idx = torch.empty(H, W, device=dev, dtype=torch.int32)
    if total < 1:  # nothing reaches 1/255 anywhere: T = 1 at every pixel (gsplat's normal path, alpha 0)
        out = background.reshape(1, 1, -1).expand(H, W, background.shape[0]).contiguous()
        final_Ts.fill_(1.0)
        final_idx.zero_()
        return (out, torch.zeros(H, W, device=dev), final_Ts, final_idx,
                torch.zeros(0, device=dev, dtype=torch.int32), torch.zeros(num_tiles, 2, device=dev, dtype=torch.int32))
    isect = torch.empty(total, device=dev, dtype=torch.int64)
    gids = torch.empty(total, device=dev, dtype=torch.int32)
    call("sfx_isect_emit_cull_views", n, n, ptr(xys), ptr(conics), ptr(opacity), ptr(depths), ptr(radii), ptr(cum),
         tiles_x, tiles_y, 16, H, W, ptr(isect), ptr(gids), None, total, stream())
    isect_s, gids_s = torch.empty_like(isect), torch.empty_like(gids)
    ws = _lib.workspace(_lib.fn("sfx_sort_workspace_bytes")(total), dev)
    call("sfx_sort_pairs_u64", total, ptr(isect), ptr(gids), ptr(isect_s), ptr(gids_s), 0,
         32 + max(1, int(num_tiles - 1).bit_length()), ptr(ws), ws.numel(), stream())
    tile_bins = torch.empty(num_tiles, 2, device=dev, dtype=torch.int32)
    call("sfx_tile_bins", total, ptr(isect_s), num_tiles, ptr(tile_bins), stream())
    rec = torch.empty(n, 16, device=dev, dtype=torch.float32)
    call("sfx_pack_raster_records", n, ptr(xys), ptr(conics), ptr(colors), ptr(opacity), ptr(rec), stream())
    out = torch.empty(H, W, 3, device=dev, dtype=torch.float32)
    alpha = torch.empty(H, W, device=dev, dtype=torch.float32)
    call("sfx_rasterize_fwd_views_quad", 1, tiles_x, tiles_y, 16, H, W, ptr(gids_s), ptr(tile_bins), ptr(rec),
         ptr(background), 0, ptr(final_Ts), ptr(final_idx), ptr(out), ptr(alpha), stream())
    return out, alpha, final_Ts, final_idx, gids_s, tile_bins


def rasterize_gaussians(xys: Tensor, depths: Tensor, radii: Tensor, conics: Tensor, num_tiles_hit: Tensor,
                        colors: Tensor, opacity: Tensor, img_height: int, img_width: int, block_width: int,
                        background: Optional[Tensor] = None, return_alpha: Optional[bool] = False):
    """Front-to-back tile rasterizer (3-channel), gsplat v0.1.11 contract: out_img [H,W,3] (+ alpha [H,W])."""
    assert block_width > 1 and block_width <= 16, "block_width must be between 2 and 16"
    if colors.dtype == torch.uint8:
        colors = colors.float() / 255
    if colors.shape[-1] != 3:
        raise NotImplementedError("only the 3-channel rasterizer is on the SplatFormer path")
    if background is not None:
        assert background.shape[0] == colors.shape[-1], \
            f"incorrect shape of background color tensor, expected shape {colors.shape[-1]}"
    else:
        background = torch.ones(colors.shape[-1], dtype=torch.float32, device=colors.device)
    if xys.ndimension() != 2 or xys.size(1) != 2:
        raise ValueError("xys must have dimensions (N, 2)")
    if colors.ndimension() != 2:
        raise ValueError("colors must have dimensions (N, D)")
    return _RasterizeGaussians.apply(xys.contiguous(), depths.contiguous(), radii.contiguous(), conics.contiguous(),
                                     num_tiles_hit.contiguous(), colors.contiguous(), opacity.contiguous(),
                                     img_height, img_width, block_width, background.contiguous(), return_alpha)
