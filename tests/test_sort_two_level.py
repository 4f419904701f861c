"""The two-level intersection sort of the culled eval render (gs_render.SORT_TWO_LEVEL, include/sfx.h
sfx_depth_keys) restated in numpy: Gaussian-views stable-argsorted by depth bits, their pairs emitted in that order,
then a stable sort of the tile bits alone -- against gsplat's one-level stable sort of the (tile << 32 | depth) keys
in emission (index) order (utils/gs_utils.py:96 -> gsplat v0.1.11 rasterize_gaussians: map_gaussian_to_intersects + sort).  Same (key, Gaussian) list,
ties included (equal depth bits in one tile keep index order).  The GPU path is checked key for key against the
oracle in tests/test_gpu_full.py."""
import numpy as np
import pytest


def one_level(tiles_of, depth_bits):
    keys, gids = [], []
    for g, tl in enumerate(tiles_of):  # emission: Gaussian-views in index order, tiles in walk order
        for t in tl:
            keys.append((t << 32) | int(depth_bits[g]))
            gids.append(g)
    keys, gids = np.array(keys, np.uint64), np.array(gids, np.int64)
    o = np.argsort(keys, kind="stable")
    return keys[o], gids[o]


def two_level(tiles_of, depth_bits):
    order = np.argsort(depth_bits, kind="stable")  # sfx_depth_keys + 4 LSD passes over 32 bits
    keys, gids = [], []
    for g in order:  # emission in depth order (sfx_isect_emit_cull_views with the depth rank)
        for t in tiles_of[g]:
            keys.append((t << 32) | int(depth_bits[g]))
            gids.append(g)
    keys, gids = np.array(keys, np.uint64), np.array(gids, np.int64)
    o = np.argsort(keys >> np.uint64(32), kind="stable")  # the tile bits only
    return keys[o], gids[o]


@pytest.mark.parametrize("seed", range(6))
def test_two_level_equals_one_level(seed):
    rng = np.random.default_rng(seed)
    n, T = 3000, 400
    # few distinct depths (ties inside tiles), some Gaussians without tiles, clustered footprints
    depth_bits = rng.integers(0, 40 if seed % 2 else 1 << 30, n).astype(np.uint32)
    tiles_of = []
    for _ in range(n):
        k = int(rng.integers(0, 6))
        t0 = int(rng.integers(0, T - 8))
        tiles_of.append(sorted(set(int(t0 + x) for x in rng.integers(0, 8, k))))
    k1, g1 = one_level(tiles_of, depth_bits)
    k2, g2 = two_level(tiles_of, depth_bits)
    assert np.array_equal(k1, k2) and np.array_equal(g1, g2)
