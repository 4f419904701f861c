"""TEST INFRASTRUCTURE ONLY (imported by tests/ as the checker, never by the product path).

CPU restatement of the fork's point-downsampling experiments, reference models/pcd_downsampling_methods.py:
furthest_point_sampling :8-26, fps_knn_downsample :29-71, map_to_original_from_centroids :74-84,
voxel_downsample :86-130, voxel_downsample_map_logits_to_original :132-161, random_downsample :164-180,
knn_map_back :182-198.  numpy fp32 arithmetic in the reference's operation order (index_add_ on the CPU sums in
index order); the 1-NN queries use the same third-party algorithm as the reference (scikit-learn
NearestNeighbors, unpinned in requirements.txt); the random draws use torch's CPU generator exactly as the
reference does.  Pinned by tests/golden/downsample.npz, captured from the reference module itself
(tests/golden/make_golden_downsample.py).
"""
from __future__ import annotations

import numpy as np
import torch
from sklearn.neighbors import NearestNeighbors


def _segment_means(n_out: int, inv: np.ndarray, *arrays):
    counts = np.zeros(n_out, np.float32)
    np.add.at(counts, inv, np.float32(1))
    outs = []
    for a in arrays:
        s = np.zeros((n_out, a.shape[1]), np.float32)
        for i in range(a.shape[0]):  # index order, like index_add_ on the CPU
            s[inv[i]] += a[i]
        outs.append(s / counts[:, None])
    return outs


def voxel_ids(points: np.ndarray, voxel_size: float) -> np.ndarray:
    vc = np.floor(points.astype(np.float32) / np.float32(voxel_size)).astype(np.int32)
    with np.errstate(over="ignore"):
        return vc[:, 0] * np.int32(1_000_000) + vc[:, 1] * np.int32(1_000) + vc[:, 2]


def voxel_downsample(points, features, grid_coords, voxel_size):
    ids = voxel_ids(points, voxel_size)
    uniq, inv = np.unique(ids, return_inverse=True)
    p, f, g = _segment_means(len(uniq), inv, points.astype(np.float32), features.astype(np.float32),
                             grid_coords.astype(np.float32))
    return p, f, np.round(g).astype(np.int64), inv


def voxel_downsample_map_logits_to_original(points, downsampled_points, logits, voxel_size):
    orig = voxel_ids(points, voxel_size)
    down = voxel_ids(downsampled_points, voxel_size)
    id_to_index = {int(v): i for i, v in enumerate(down)}
    return logits[np.array([id_to_index[int(v)] for v in orig])]


def furthest_point_sampling(xyz: np.ndarray, npoint: int, start: int) -> np.ndarray:
    xyz = xyz.astype(np.float32)
    centroids = np.zeros(npoint, np.int64)
    distance = np.full(xyz.shape[0], np.float32(1e10), np.float32)
    farthest = start
    for i in range(npoint):
        centroids[i] = farthest
        d = xyz - xyz[farthest]
        d = d * d
        dist = (d[:, 0] + d[:, 1]) + d[:, 2]
        np.minimum(distance, dist, out=distance, where=dist < distance)
        farthest = int(np.argmax(distance))  # first maximum
    return centroids


def fps_start(n: int) -> int:
    """The reference's start draw: torch.randint(0, N, (1,)).item() on the current CPU generator."""
    return int(torch.randint(0, n, (1,)).item())


def nn1(queries: np.ndarray, refs: np.ndarray) -> np.ndarray:
    nbrs = NearestNeighbors(n_neighbors=1, algorithm="auto").fit(refs)
    return nbrs.kneighbors(queries)[1][:, 0]


def fps_knn_downsample(points, features, grid_coords, ratio, start):
    N = points.shape[0]
    M = int(N * ratio)
    cidx = furthest_point_sampling(points, M, start)
    assign = nn1(points, points[cidx])
    p, f, g = _segment_means(M, assign, points.astype(np.float32), features.astype(np.float32),
                             grid_coords.astype(np.float32))
    return p, f, np.round(g).astype(np.int64), assign, cidx


def random_indices(n: int, ratio: float) -> np.ndarray:
    """torch.randperm(N)[:M] on the current CPU generator (random_downsample :176)."""
    return torch.randperm(n)[:int(n * ratio)].numpy()


def knn_map_back(processed, sampled_points, original_points):
    return processed[nn1(original_points, sampled_points)]
