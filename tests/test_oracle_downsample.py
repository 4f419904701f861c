"""oracle/downsample_ref.py against golden vectors captured from the reference's own
models/pcd_downsampling_methods.py (tests/golden/make_golden_downsample.py)."""
import os

import numpy as np
import torch

from oracle import downsample_ref as D

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "downsample.npz"))


def test_voxel_downsample_golden():
    p, f, g, inv = D.voxel_downsample(G["points"], G["feat"], G["grid"], float(G["voxel_size"]))
    assert np.array_equal(p, G["vox_points"]) and np.array_equal(f, G["vox_feat"])
    assert np.array_equal(g, G["vox_grid"])
    mapped = D.voxel_downsample_map_logits_to_original(G["points"], p, G["vox_logits"], float(G["voxel_size"]))
    assert np.array_equal(mapped, G["vox_mapped"])
    assert np.array_equal(G["vox_logits"][inv], G["vox_mapped"])  # the cluster id is the reference's map


def test_random_downsample_golden():
    torch.manual_seed(int(G["rnd_seed"]))
    idx = D.random_indices(G["points"].shape[0], float(G["rnd_ratio"]))
    assert np.array_equal(idx, G["rnd_idx"])
    assert np.array_equal(G["points"][idx], G["rnd_points"])
    mapped = D.knn_map_back(G["rnd_logits"], G["rnd_points"], G["points"])
    assert np.array_equal(mapped, G["rnd_mapped"])


def test_fps_golden():
    torch.manual_seed(int(G["fps_seed"]))
    start = D.fps_start(G["points"].shape[0])
    cidx = D.furthest_point_sampling(G["points"], 300, start)
    assert np.array_equal(cidx, G["fps_centroids"])
    p, f, g, a, _ = D.fps_knn_downsample(G["points"], G["feat"], G["grid"], float(G["fps_ratio"]), start)
    assert np.array_equal(a, G["fps_assign"])
    assert np.array_equal(p, G["fps_points"]) and np.array_equal(f, G["fps_feat"])
    assert np.array_equal(g, G["fps_grid"])
