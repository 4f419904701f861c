"""Point-cloud downsampling experiments of the fork, device-side.

Mirrors reference models/pcd_downsampling_methods.py (same names, arguments and return values) and its use in
FeaturePredictor (models/feature_predictor.py:159-196, `additional_info["downsample"]` in {"voxel", "fps",
"random"}):

* `voxel_downsample` (:86-130): voxel keys (`sfx_voxel_keys`) -> stable radix sort -> run flags + scan ->
  clusters (`sfx_pool_run_flags` / `sfx_pool_assign_runs`, the sort-free pooling kernels) -> per-voxel means of
  points, features and grid coordinates (`sfx_segment_mean`, summed in index order), grid means rounded.
* `voxel_downsample_map_logits_to_original` (:132-161): the voxel of every original point (the reference
  rebuilds it from floor(mean / voxel_size) through a Python dict; the mean of a voxel's points lies in that
  voxel, so this is the cluster id -- identical whenever the reference's dict lookup succeeds).
* `furthest_point_sampling` (:8-26): `sfx_fps` from the same `torch.randint` start draw.
* `fps_knn_downsample` (:29-71): FPS + 1-NN assignment (`sfx_nn1`, the sklearn query) + per-centroid means.
* `random_downsample` (:164-180): the same `torch.randperm` draw (host RNG), gathered on the device.
* `knn_map_back` (:182-198): `sfx_nn1` from every original point to the sampled points.

Parity: tests/golden/downsample.npz (captured from the reference module itself, tests/golden/
make_golden_downsample.py) and oracle/downsample_ref.py; tests/test_gpu_downsample.py.
"""
from __future__ import annotations

import torch
from torch import Tensor

from . import _lib
from . import ptv3_ops as ops
from ._lib import I, L, P, F, call, ptr, stream

_lib.register("sfx_voxel_keys", [I, P, L, F, P, P])
_lib.register("sfx_nn1", [I, I, P, P, P, P])
_lib.register("sfx_fps", [I, I, P, I, P, P, P])


def _xyz(t: Tensor) -> Tensor:
    return t.float().contiguous()


def _clusters(keys: Tensor):
    """Stable sort of u64 keys -> (sorted member list, cluster id per point, CSR pointers, cluster count)."""
    n = keys.shape[0]
    _, order = ops._sort(keys, None, 0, 32)
    flags = torch.empty(n, device=keys.device, dtype=torch.int32)
    call("sfx_pool_run_flags", n, 1, ptr(order), ptr(keys.view(torch.int64)), 0, ptr(flags), stream())
    pos, total = ops.scan_i32(flags)
    m = int(total.item())
    cluster = torch.empty(n, device=keys.device, dtype=torch.int32)
    sidx = torch.empty(n, device=keys.device, dtype=torch.int32)
    idx_ptr = torch.empty(m + 1, device=keys.device, dtype=torch.int32)
    head = torch.empty(m, device=keys.device, dtype=torch.int32)
    call("sfx_pool_assign_runs", n, m, 0, ptr(order), ptr(pos), ptr(flags), ptr(cluster), ptr(idx_ptr), ptr(head),
         ptr(sidx), stream())
    return sidx, cluster, idx_ptr, m


def _means(points: Tensor, features: Tensor, grid_coords: Tensor, idx_ptr: Tensor, sidx: Tensor, m: int):
    p = ops.segment_mean(_xyz(points), idx_ptr, sidx, m)
    f = ops.segment_mean(features.float().contiguous(), idx_ptr, sidx, m)
    g = ops.segment_mean(grid_coords.float().contiguous(), idx_ptr, sidx, m)
    return p, f, g.round().long()


def voxel_downsample_with_inverse(points: Tensor, features: Tensor, grid_coords: Tensor, voxel_size: float):
    """voxel_downsample plus the voxel (cluster id, int32) of every input point."""
    assert points.shape[0] == features.shape[0]
    _lib.require_gpu(points)
    n = points.shape[0]
    keys = torch.empty(n, device=points.device, dtype=torch.int64)
    pts = _xyz(points)
    call("sfx_voxel_keys", n, ptr(pts), pts.stride(0), float(voxel_size), ptr(keys), stream())
    sidx, cluster, idx_ptr, m = _clusters(keys)
    return (*_means(points, features, grid_coords, idx_ptr, sidx, m), cluster)


def voxel_downsample(points: Tensor, features: Tensor, grid_coords: Tensor, voxel_size: float):
    """-> (downsampled points [M,3], features [M,C], grid coords [M,3] long)."""
    return voxel_downsample_with_inverse(points, features, grid_coords, voxel_size)[:3]


def voxel_downsample_map_logits_to_original(points: Tensor, downsampled_points: Tensor, logits: Tensor,
                                            voxel_size: float, inverse: Tensor = None) -> Tensor:
    if inverse is None:  # the voxels of the original points (same keys, same stable clusters)
        z = torch.zeros(points.shape[0], 1, device=points.device)
        inverse = voxel_downsample_with_inverse(points, z, z, voxel_size)[3]
    return logits.index_select(0, inverse.long())


def furthest_point_sampling(xyz: Tensor, npoint: int, start: int = None) -> Tensor:
    """Indices of `npoint` furthest-point picks; `start` (the first pick) is drawn as the reference draws it
    when None (tests pass the golden's first pick to pin the deterministic part)."""
    _lib.require_gpu(xyz)
    N = xyz.shape[0]
    if N == 0 or npoint <= 0:
        raise ValueError(f"furthest_point_sampling: need N > 0 and npoint > 0 (got N={N}, npoint={npoint})")
    # the reference's draw on the points' device (pcd_downsampling_methods.py:17): the device generator, as the
    # reference's GPU run does; parity of this device draw against a CUDA run is unpinned (the goldens are CPU)
    if start is None:
        start = int(torch.randint(0, N, (1,), device=xyz.device).item())
    if not 0 <= start < N:
        raise ValueError(f"furthest_point_sampling: start {start} out of range [0, {N})")
    pts = _xyz(xyz)
    out = torch.empty(npoint, device=xyz.device, dtype=torch.int32)
    ws = torch.empty(N, device=xyz.device, dtype=torch.float32)
    call("sfx_fps", N, npoint, ptr(pts), start, ptr(out), ptr(ws), stream())
    return out.long()


def nn1(queries: Tensor, refs: Tensor) -> Tensor:
    """Index of the nearest reference point for every query (the sklearn 1-NN query of the reference)."""
    q, r = _xyz(queries), _xyz(refs)
    if r.shape[0] == 0 and q.shape[0] > 0:
        raise ValueError("nn1: empty reference set (a downsampling ratio that keeps no point)")
    out = torch.empty(q.shape[0], device=q.device, dtype=torch.int32)
    call("sfx_nn1", q.shape[0], r.shape[0], ptr(q), ptr(r), ptr(out), stream())
    return out


def fps_knn_downsample(points: Tensor, features: Tensor, grid_coords: Tensor, ratio: float, start: int = None):
    """-> (points [M,3], features [M,C], grid coords [M,3] long, assignments [N] long)."""
    N = points.shape[0]
    M = int(N * ratio)
    if M <= 0:
        raise ValueError(f"fps_knn_downsample: int(N * ratio) = {M} keeps no point (N={N}, ratio={ratio})")
    centroid_idx = furthest_point_sampling(points, M, start)
    centroids = points[centroid_idx]
    assignments = nn1(points, centroids)
    keys = assignments.to(torch.int64)
    sidx, _, idx_ptr, m = _clusters(keys)
    if m != M:  # a centroid no point is nearest to (only with duplicated positions): reference divides by 0
        raise RuntimeError(f"fps_knn_downsample: {M - m} centroids received no point")
    p, f, g = _means(points, features, grid_coords, idx_ptr, sidx, m)
    return p, f, g, assignments.long()


def map_to_original_from_centroids(downsampled_features: Tensor, assignments: Tensor) -> Tensor:
    return downsampled_features[assignments]


def random_downsample(points: Tensor, features: Tensor, grid_coord: Tensor, ratio: float):
    N = points.shape[0]
    M = int(N * ratio)
    if M <= 0:
        raise ValueError(f"random_downsample: int(N * ratio) = {M} keeps no point (N={N}, ratio={ratio})")
    indices = torch.randperm(N)[:M].to(points.device)  # the reference's host draw
    return points[indices], features[indices], grid_coord[indices], indices


def knn_map_back(processed_features: Tensor, sampled_points: Tensor, original_points: Tensor) -> Tensor:
    return processed_features[nn1(original_points, sampled_points).long()]


def downsample_for_backbone(method: str, info: dict, coord: Tensor, feat: Tensor, grid: Tensor):
    """FeaturePredictor's downsample branch (feature_predictor.py:159-171) -> (coord, feat, grid int32, mapper)
    where mapper(y) maps the backbone output of the downsampled points back to the originals (:186-196)."""
    if method == "voxel":
        vs = info["voxel_size"]
        c, f, g, inv = voxel_downsample_with_inverse(coord, feat, grid, vs)
        return c, f, g.int(), lambda y: voxel_downsample_map_logits_to_original(coord, c, y, vs, inverse=inv)
    if method == "fps":
        c, f, g, a = fps_knn_downsample(coord, feat, grid, info["downsample_ratio"])
        return c, f, g.int(), lambda y: map_to_original_from_centroids(y, a)
    if method == "random":
        c, f, g, _ = random_downsample(coord, feat, grid, info["downsample_ratio"])
        return c.contiguous(), f.contiguous(), g.int().contiguous(), lambda y: knn_map_back(y, c, coord)
    raise NotImplementedError(method)
