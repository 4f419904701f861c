"""Render glue: mirror of reference utils/gs_utils.py:12-114.

`rasterize_gaussians_to_singleimg` / `rasterize_gaussians_to_multiimgs` keep the
reference signatures (gs_utils.py:20, :29).  Two device paths, both HIP:

* eval (no autograd needed): one fused kernel `sfx_render_prep_project`
  (viewmat, exp/normalise/sigmoid, SH, EWA projection) followed by the
  device scan / radix sort / tile rasterizer -- no torch elementwise ops and
  no `.item()` on the camera (intrinsics are taken as host scalars).
* training (params require grad): the reference's torch glue around the
  autograd Functions of `gsplat_compat` so gradients flow to the refined
  Gaussians (reference train.py:273-289).
"""
from __future__ import annotations

import math
from typing import Dict, List, Tuple

import torch
from torch import Tensor

from . import _lib
from . import ptv3_ops as ops
from ._lib import F, I, L, P, call, ptr, stream
from .gsplat_compat import (_RasterizeGaussians, bin_and_sort_gaussians, compute_cumulative_intersects,
                            project_gaussians, rasterize_gaussians, spherical_harmonics)

BLOCK_WIDTH = 16
# eval path: exact contribution culling + per-wave quadrant lists (ABI v9).  Images, alphas and final T are
# bit-identical either way; SFX_RENDER_CULL=0 restores gsplat's full 3-sigma intersection list (the list the
# intersection-level parity tests compare key for key).
import os as _os
RENDER_CULL = _os.environ.get("SFX_RENDER_CULL", "1") != "0"
# culled eval path: two-level intersection sort (depth argsort of the Gaussian-views, then the tile bits of the
# depth-ordered pairs); SFX_SORT_TWO_LEVEL=0: one radix sort of all 32 + tile bits of every pair
SORT_TWO_LEVEL = _os.environ.get("SFX_SORT_TWO_LEVEL", "1") != "0"
C0 = 0.28209479177387814


def SH2RGB(sh):
    return sh * C0 + 0.5


def RGB2SH(rgb):
    return (rgb - 0.5) / C0


def _scalar(x) -> float:
    return float(x.item()) if isinstance(x, Tensor) else float(x)


_lib.register("sfx_render_prep_project_views", [I, I, I, P, L, P, L, P, L, P, L, P, L, P, L, P, F, F, F, F, I, I, I,
                                                 P, P, P, P, P, P, P, P, P])
_lib.register("sfx_isect_emit_views", [I, I, P, P, P, P, I, I, I, P, P, L, P])
_lib.register("sfx_rasterize_fwd_views", [I, I, I, I, I, I, P, P, P, P, P, P, P, I, P, P, P, P, P])
_lib.register("sfx_pack_raster_records", [I, P, P, P, P, P, P])
_lib.register("sfx_rasterize_fwd_views_packed", [I, I, I, I, I, I, P, P, P, P, I, P, P, P, P, P])
_lib.register("sfx_isect_count_cull_views", [I, I, P, P, P, P, I, I, I, I, I, P, P])
_lib.register("sfx_isect_emit_cull_views", [I, I, P, P, P, P, P, P, I, I, I, I, I, P, P, P, L, P])
_lib.register("sfx_depth_keys", [L, P, P, P])
_lib.register("sfx_invert_permutation", [L, P, P, P])
_lib.register("sfx_rasterize_fwd_views_quad", [I, I, I, I, I, I, P, P, P, P, I, P, P, P, P, P])


def rasterize_gaussians_to_multiimgs(gs_params: Dict[str, Tensor], cameras: Dict) -> Tuple[List[Tensor], List[Tensor]]:
    """gs_utils.py:20-27: render every camera_to_world of `cameras`.

    Eval (no autograd): all views in one batched pass -- one fused prep/project launch for V cameras, one
    scan, one stable radix sort of every view's (view, tile, depth) keys, one rasterizer launch over
    V x tiles -- per-view results identical to rendering the views one by one.  Training: per view through
    the autograd glue, as the reference."""
    gp = {k: v.float() if v.dtype == torch.half else v for k, v in gs_params.items()}
    c2ws = cameras["camera_to_worlds"]
    if len(c2ws) > 1 and not _needs_grad(gp) and "opacities_sigmoid" not in gp and "opacities" in gp:
        return _render_fused_views(gp, c2ws, cameras)
    rgbs, alphas = [], []
    prep = views = None
    if _needs_grad(gp) or "opacities_sigmoid" in gp:  # training: the view-independent glue once per scene
        if "opacities" not in gp and "opacities_sigmoid" not in gp:
            raise ValueError("No opacities found in gs_params")
        prep = _autograd_prep(gp)
        c2w_all = c2ws if isinstance(c2ws, Tensor) else torch.stack(list(c2ws))
        views = _autograd_views(prep[0], c2w_all)
    for v, camera_to_world in enumerate(cameras["camera_to_worlds"]):
        rgb, alpha = rasterize_gaussians_to_singleimg(gs_params, camera_to_world, _prep=prep,
                                                      _view=None if views is None else (views[0][v], views[1][v]),
                                                      **cameras)
        rgbs.append(rgb)
        alphas.append(alpha)
    return rgbs, alphas


def _needs_grad(gs_params) -> bool:
    return torch.is_grad_enabled() and any(isinstance(v, Tensor) and v.requires_grad for v in gs_params.values())


def rasterize_gaussians_to_singleimg(gs_params, camera_to_world, cx, cy, fx, fy, width, height, background_color,
                                     _prep=None, _view=None, **kwargs):
    """gs_utils.py:29-114 -> (rgb [H,W,3] clamped <= 1, alpha [H,W,1])."""
    gs_params = {k: v.float() if v.dtype == torch.half else v for k, v in gs_params.items()}
    if "opacities" not in gs_params and "opacities_sigmoid" not in gs_params:
        raise ValueError("No opacities found in gs_params")
    H, W = int(_scalar(height)), int(_scalar(width))
    fx, fy, cx, cy = _scalar(fx), _scalar(fy), _scalar(cx), _scalar(cy)
    if _needs_grad(gs_params) or "opacities_sigmoid" in gs_params:
        return _render_autograd(gs_params, camera_to_world, cx, cy, fx, fy, W, H, background_color, prep=_prep,
                                view=_view)
    return _render_fused(gs_params, camera_to_world, cx, cy, fx, fy, W, H, background_color)


def _rowptr(t: Tensor, width: int):
    """(pointer, row stride) of an [N, ...] attribute whose per-row `width` floats are contiguous."""
    t2 = t.reshape(t.shape[0], -1) if t.is_contiguous() else t
    if t2.dim() == 3:  # e.g. features_rest view [N, K, 3] of a packed record
        if t2.stride(2) == 1 and t2.stride(1) == 3:
            return t2.data_ptr(), t2.stride(0), t2
        t2 = t2.contiguous().reshape(t.shape[0], -1)
    if t2.dim() == 2 and t2.stride(1) == 1 and t2.shape[1] == width:
        return t2.data_ptr(), t2.stride(0), t2
    t2 = t.contiguous().reshape(t.shape[0], -1)
    return t2.data_ptr(), t2.stride(0), t2


def _render_fused(gs, c2w, cx, cy, fx, fy, W, H, background):
    means = gs["means"]
    _lib.require_gpu(means)
    dev = means.device
    n = means.shape[0]
    rest = gs.get("features_rest")
    nb = 1 + (rest.shape[1] if rest is not None else 0)
    keep = []
    pm, lm, t = _rowptr(means, 3); keep.append(t)
    ps, ls, t = _rowptr(gs["scales"], 3); keep.append(t)
    pq, lq, t = _rowptr(gs["quats"], 4); keep.append(t)
    po, lo, t = _rowptr(gs["opacities"], 1); keep.append(t)
    pd, ldc, t = _rowptr(gs["features_dc"], 3); keep.append(t)
    pr, lr = None, 0
    if rest is not None:
        pr, lr, t = _rowptr(rest, 3 * (nb - 1)); keep.append(t)
    c2w = c2w.detach().float().contiguous()
    f = lambda *s, dt=torch.float32: torch.empty(*s, device=dev, dtype=dt)
    viewmat, rgbs, opac = f(3, 4), f(n, 3), f(n, 1)
    xys, depths, radii, conics, tiles = f(n, 2), f(n), f(n, dt=torch.int32), f(n, 3), f(n, dt=torch.int32)
    call("sfx_render_prep_project", n, nb, pm, lm, ps, ls, pq, lq, po, lo, pd, ldc, pr, lr, ptr(c2w), fx, fy, cx, cy,
         H, W, BLOCK_WIDTH, ptr(viewmat), ptr(rgbs), ptr(opac), ptr(xys), ptr(depths), ptr(radii), ptr(conics),
         ptr(tiles), stream())
    bg = background.to(device=dev, dtype=torch.float32).contiguous()
    rgb, alpha = _RasterizeGaussians.apply(xys, depths, radii, conics, tiles, rgbs, opac, H, W, BLOCK_WIDTH, bg, True)
    rgb = torch.clamp(rgb, max=1.0)
    return rgb, alpha.unsqueeze(-1)


def render_views_meta(gs_params: Dict[str, Tensor], cameras: Dict):
    """The batched eval path of rasterize_gaussians_to_multiimgs, also returning its intermediate device buffers
    (per-view projection records, intersection keys / ids after the sort, tile bins) for parity checks and
    tools.  -> (rgbs, alphas, meta)."""
    gp = {k: v.float() if v.dtype == torch.half else v for k, v in gs_params.items()}
    meta: Dict = {}
    rgbs, alphas = _render_fused_views(gp, cameras["camera_to_worlds"], cameras, meta=meta)
    return rgbs, alphas, meta


def _render_fused_views(gs, c2ws, cameras, meta=None):
    means = gs["means"]
    _lib.require_gpu(means)
    dev = means.device
    n = means.shape[0]
    V = int(c2ws.shape[0])
    H, W = int(_scalar(cameras["height"])), int(_scalar(cameras["width"]))
    fx, fy, cx, cy = (_scalar(cameras[k]) for k in ("fx", "fy", "cx", "cy"))
    bg = cameras["background_color"].to(device=dev, dtype=torch.float32).contiguous()
    rest = gs.get("features_rest")
    nb = 1 + (rest.shape[1] if rest is not None else 0)
    keep = []
    pm, lm, t = _rowptr(means, 3); keep.append(t)
    ps, ls, t = _rowptr(gs["scales"], 3); keep.append(t)
    pq, lq, t = _rowptr(gs["quats"], 4); keep.append(t)
    po, lo, t = _rowptr(gs["opacities"], 1); keep.append(t)
    pd, ldc, t = _rowptr(gs["features_dc"], 3); keep.append(t)
    pr, lr = None, 0
    if rest is not None:
        pr, lr, t = _rowptr(rest, 3 * (nb - 1)); keep.append(t)
    cams = c2ws.detach().to(device=dev, dtype=torch.float32).contiguous()
    f = lambda *s, dt=torch.float32: torch.empty(*s, device=dev, dtype=dt)
    rgbs, opac, xys, depths = f(V, n, 3), f(V, n), f(V, n, 2), f(V, n)
    radii, conics, tiles = f(V, n, dt=torch.int32), f(V, n, 3), f(V * n, dt=torch.int32)
    call("sfx_render_prep_project_views", n, V, nb, pm, lm, ps, ls, pq, lq, po, lo, pd, ldc, pr, lr, ptr(cams), fx, fy,
         cx, cy, H, W, BLOCK_WIDTH, ptr(rgbs), ptr(opac), ptr(xys), ptr(depths), ptr(radii), ptr(conics), ptr(tiles),
         None, stream())
    # inclusive scan of the tiles hit; the per-view ends (and the total = the last of them) reach the host in ONE
    # asynchronous read, with the count-independent record packing enqueued in front of the wait (a separate pass:
    # writing the records from the prep measured slower, 186 vs 106 + 69 us at config E)
    cum = torch.empty(V * n, device=dev, dtype=torch.int32)
    rec = f(V * n, 16)  # packed 64-byte records: one gather per Gaussian in the rasterizer's batch fetch
    bw = BLOCK_WIDTH
    tiles_x, tiles_y = (W + bw - 1) // bw, (H + bw - 1) // bw
    T = tiles_x * tiles_y
    cull = RENDER_CULL and bw == 16
    kept = tiles
    if n:
        if cull:  # surviving tile counts (gsplat's 3-sigma counts stay in `tiles`)
            kept = torch.empty(V * n, device=dev, dtype=torch.int32)
            call("sfx_isect_count_cull_views", V * n, n, ptr(xys), ptr(conics), ptr(opac), ptr(radii), tiles_x,
                 tiles_y, bw, H, W, ptr(kept), stream())
        tot_dev = torch.empty(1, device=dev, dtype=torch.int32)
        ws = _lib.workspace(_lib.fn("sfx_scan_workspace_bytes")(V * n), dev)
        call("sfx_scan_i32", V * n, ptr(kept), ptr(cum), 1, ptr(ws), ws.numel(), ptr(tot_dev), stream())
        ends_rd = _lib.HostRead(cum.view(V, n)[:, -1])
        call("sfx_pack_raster_records", V * n, ptr(xys), ptr(conics), ptr(rgbs), ptr(opac), ptr(rec), stream())
        if cull and SORT_TWO_LEVEL:
            # two-level sort (include/sfx.h sfx_depth_keys): the Gaussian-views argsorted by depth (4 passes over
            # V n keys), their surviving tile counts scanned in that order -- queued while the host waits for `ends`
            dkeys = torch.empty(V * n, device=dev, dtype=torch.int64)
            call("sfx_depth_keys", V * n, ptr(depths), ptr(dkeys), stream())
            _, dorder = ops._sort(dkeys, None, 0, 32)
            del dkeys
            drank = torch.empty_like(dorder)
            call("sfx_invert_permutation", V * n, ptr(dorder), ptr(drank), stream())
            cum_o = torch.empty(V * n, device=dev, dtype=torch.int32)
            call("sfx_scan_i32", V * n, ptr(kept.index_select(0, dorder)), ptr(cum_o), 1, ptr(ws), ws.numel(),
                 ptr(tot_dev), stream())
        ends = ends_rd.get()
    else:
        ends = [0] * V
    total = ends[-1]
    # per-view intersection counts (gsplat's empty-image branch is per call: alpha = 1 there)
    per_view = [ends[0]] + [ends[v] - ends[v - 1] for v in range(1, V)]
    if cull and n and not all(per_view):  # rare: a view kept nothing -- is gsplat's own list empty too?
        full = tiles.view(V, n).sum(1, dtype=torch.int64).tolist()
        per_view = [max(c, int(f)) for c, f in zip(per_view, full)]
    out = f(V, H, W, 3)
    alpha = f(V, H, W)
    if total > 0:
        isect = f(total, dt=torch.int64)
        gids = f(total, dt=torch.int32)
        two_level = cull and SORT_TWO_LEVEL
        if cull:
            call("sfx_isect_emit_cull_views", V * n, n, ptr(xys), ptr(conics), ptr(opac), ptr(depths), ptr(radii),
                 ptr(cum_o if two_level else cum), tiles_x, tiles_y, bw, H, W, ptr(isect), ptr(gids),
                 ptr(drank) if two_level else None, total, stream())
        else:
            call("sfx_isect_emit_views", V * n, n, ptr(xys), ptr(depths), ptr(radii), ptr(cum), tiles_x, tiles_y, bw,
                 ptr(isect), ptr(gids), total, stream())
        isect_s, gids_s = torch.empty_like(isect), torch.empty_like(gids)
        key_bits = 32 + max(1, int(V * T - 1).bit_length())
        ws = _lib.workspace(_lib.fn("sfx_sort_workspace_bytes")(total), dev)
        # two-level: the pairs arrive depth-sorted, so a stable sort of the tile bits alone finishes gsplat's order
        call("sfx_sort_pairs_u64", total, ptr(isect), ptr(gids), ptr(isect_s), ptr(gids_s), 32 if two_level else 0,
             key_bits, ptr(ws), ws.numel(), stream())
        del isect, gids
        bins = f(V * T, 2, dt=torch.int32)
        call("sfx_tile_bins", total, ptr(isect_s), V * T, ptr(bins), stream())
        final_Ts, final_idx = f(V, H, W), f(V, H, W, dt=torch.int32)
        call("sfx_rasterize_fwd_views_quad" if cull else "sfx_rasterize_fwd_views_packed", V, tiles_x, tiles_y, bw,
             H, W, ptr(gids_s), ptr(bins), ptr(rec), ptr(bg), 1, ptr(final_Ts), ptr(final_idx), ptr(out),
             ptr(alpha), stream())
    elif any(c > 0 for c in per_view):  # every gsplat intersection culled: T = 1 at every pixel of those views
        out[:] = torch.clamp(bg, max=1.0)
        alpha.zero_()
    for v in range(V):
        if per_view[v] < 1:
            out[v] = torch.clamp(bg, max=1.0).expand(H, W, 3)
            alpha[v] = 1.0
    if meta is not None:
        meta.update(rgbs=rgbs, opacities=opac, xys=xys, depths=depths, radii=radii, conics=conics,
                    num_tiles_hit=tiles.view(V, n), num_tiles_kept=kept.view(V, n), per_view=per_view, tiles_x=tiles_x,
                    tiles_y=tiles_y, culled=cull)
        if total > 0:
            meta.update(isect_sorted=isect_s, gids_sorted=gids_s, tile_bins=bins.view(V, T, 2), final_Ts=final_Ts,
                        final_idx=final_idx)
    return list(out.unbind(0)), list(alpha.unsqueeze(-1).unbind(0))


def _autograd_prep(gs_params):
    """The view-independent half of the reference glue (gs_utils.py:42-66): activated scales, normalised quaternions
    (rows whose norm is off by > 1e-6 -> identity, as the reference's masked assignment, via torch.where: no host
    read), opacities, SH coefficients.  Computed once per scene for all its views: the same ops, so the same values
    and, through autograd, the same summed gradients as per view."""
    means = gs_params["means"]
    scales = torch.exp(gs_params["scales"])
    quats = gs_params["quats"] / torch.norm(gs_params["quats"], dim=-1, keepdim=True)
    mask = (quats.norm(dim=-1) - 1) < 1e-6
    quats = torch.where(mask[:, None], quats, torch.tensor([0, 0, 0, 1.0], device=quats.device, dtype=quats.dtype))
    if "opacities" in gs_params:
        opacities = torch.sigmoid(gs_params["opacities"])
    else:
        opacities = gs_params["opacities_sigmoid"]
    if "features_rest" in gs_params:
        colors = torch.cat([gs_params["features_dc"].unsqueeze(1), gs_params["features_rest"]], dim=1)
    else:
        colors = gs_params["features_dc"].unsqueeze(1)
    return means, scales, quats, opacities, colors


@torch.no_grad()
def _autograd_views(means, c2ws):
    """The camera half of the glue (gs_utils.py:32-40, :70-77) for all views of a scene at once: viewmats [V, 3, 4]
    (R = c2w[:3, :3] diag(1, -1, -1) as a column sign flip, [R^T | -R^T t]) and unit view directions [V, n, 3] (zero
    norm -> (0, 0, 1)).  Neither carries a gradient (the cameras are fixed and the reference takes
    the directions from means.detach()); batched, the per-view glue is ~10 small launches shorter."""
    c2ws = c2ws.detach()
    sign = torch.tensor([1.0, -1.0, -1.0], device=c2ws.device, dtype=c2ws.dtype)
    R_inv = (c2ws[:, :3, :3] * sign).transpose(1, 2)
    T_inv = -(R_inv @ c2ws[:, :3, 3:4])
    viewmats = torch.cat([R_inv, T_inv], 2).float()
    vd = means.detach()[None] - c2ws[:, None, :3, 3]
    nrm = vd.norm(dim=-1, keepdim=True)
    vd = torch.where(nrm == 0, torch.tensor([0.0, 0.0, 1.0], device=vd.device, dtype=vd.dtype), vd / nrm)
    return viewmats, vd


def _render_autograd(gs_params, camera_to_world, cx, cy, fx, fy, W, H, background_color, prep=None, view=None):
    """Line-for-line the reference glue (gs_utils.py:32-112) over the HIP autograd ops (`prep`: _autograd_prep of
    the same Gaussians, shared by the views of a scene; `view`: this view's (viewmat, view directions) from
    _autograd_views)."""
    means, scales, quats, opacities, colors = prep if prep is not None else _autograd_prep(gs_params)
    if view is None:
        vms, vds = _autograd_views(means, camera_to_world[None])
        view = (vms[0], vds[0])
    viewmat, viewdirs = view
    n = int(math.sqrt(colors.shape[1]) - 1)
    if n == 0:
        rgbs = torch.sigmoid(colors[:, 0, :])
    else:
        rgbs = spherical_harmonics(n, viewdirs, colors)
        rgbs = torch.clamp(rgbs + 0.5, min=0.0)
    xys, depths, radii, conics, comp, num_tiles_hit, cov3d = project_gaussians(
        means, scales, 1, quats, viewmat, fx, fy, cx, cy, H, W, BLOCK_WIDTH)
    rgb, alpha = rasterize_gaussians(xys, depths, radii, conics, num_tiles_hit, rgbs, opacities, H, W, BLOCK_WIDTH,
                                     background=background_color, return_alpha=True)
    rgb = torch.clamp(rgb, max=1.0)
    alpha = alpha.unsqueeze(-1)
    return rgb, alpha


__all__ = ["rasterize_gaussians_to_multiimgs", "rasterize_gaussians_to_singleimg", "render_views_meta", "BLOCK_WIDTH", "SH2RGB", "RGB2SH",
           "bin_and_sort_gaussians", "compute_cumulative_intersects"]
