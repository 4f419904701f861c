"""HIP point-downsampling experiments (splatformer_amd/downsample.py) vs the golden vectors captured from the
reference's models/pcd_downsampling_methods.py and vs oracle/downsample_ref.py at larger sizes: index work
(voxel clusters, FPS picks, 1-NN assignments, random draws) bit-exact; the fp32 means bit-exact as well (both
sum the members in index order and divide once)."""
import os

import numpy as np
import pytest
import torch

from oracle import downsample_ref as D
from splatformer_amd import downsample as ds

pytestmark = pytest.mark.gpu
G = np.load(os.path.join(os.path.dirname(__file__), "golden", "downsample.npz"))


def dev_(a, device):
    return torch.from_numpy(np.ascontiguousarray(a)).to(device)


def test_voxel_downsample_golden(device):
    pts, feat, grid = dev_(G["points"], device), dev_(G["feat"], device), dev_(G["grid"], device)
    p, f, g = ds.voxel_downsample(pts, feat, grid, float(G["voxel_size"]))
    assert np.array_equal(p.cpu().numpy(), G["vox_points"])
    assert np.array_equal(f.cpu().numpy(), G["vox_feat"])
    assert np.array_equal(g.cpu().numpy(), G["vox_grid"])
    mapped = ds.voxel_downsample_map_logits_to_original(pts, p, dev_(G["vox_logits"], device),
                                                        float(G["voxel_size"]))
    assert np.array_equal(mapped.cpu().numpy(), G["vox_mapped"])


def test_random_downsample_golden(device):
    pts, feat, grid = dev_(G["points"], device), dev_(G["feat"], device), dev_(G["grid"], device)
    torch.manual_seed(int(G["rnd_seed"]))
    p, f, g, idx = ds.random_downsample(pts, feat, grid, float(G["rnd_ratio"]))
    assert np.array_equal(idx.cpu().numpy(), G["rnd_idx"])
    assert np.array_equal(p.cpu().numpy(), G["rnd_points"]) and np.array_equal(f.cpu().numpy(), G["rnd_feat"])
    mapped = ds.knn_map_back(dev_(G["rnd_logits"], device), p, pts)
    assert np.array_equal(mapped.cpu().numpy(), G["rnd_mapped"])


def test_fps_knn_golden(device):
    pts, feat, grid = dev_(G["points"], device), dev_(G["feat"], device), dev_(G["grid"], device)
    start = int(G["fps_centroids"][0])  # the reference's CPU draw; the product draws on the device generator
    cidx = ds.furthest_point_sampling(pts, 300, start)
    assert np.array_equal(cidx.cpu().numpy(), G["fps_centroids"])
    p, f, g, a = ds.fps_knn_downsample(pts, feat, grid, float(G["fps_ratio"]), start=start)
    assert np.array_equal(a.cpu().numpy(), G["fps_assign"])
    assert np.array_equal(p.cpu().numpy(), G["fps_points"]) and np.array_equal(f.cpu().numpy(), G["fps_feat"])
    assert np.array_equal(g.cpu().numpy(), G["fps_grid"])


@pytest.mark.parametrize("n,m", [(20000, 5000), (4097, 1), (1, 3)])
def test_nn1_vs_sklearn(device, n, m):
    rng = np.random.default_rng(n + m)
    q = rng.random((n, 3), dtype=np.float32)
    r = rng.random((m, 3), dtype=np.float32)
    got = ds.nn1(dev_(q, device), dev_(r, device)).cpu().numpy()
    assert np.array_equal(got, D.nn1(q, r))


def test_fps_vs_oracle_larger(device):
    from splatformer_amd.scenes import make_scene
    pts = make_scene(20000, 1, seed=3)["means"].float()
    torch.manual_seed(5)
    st = D.fps_start(20000)
    got = ds.furthest_point_sampling(pts.to(device), 1000, st).cpu().numpy()
    ref = D.furthest_point_sampling(pts.numpy(), 1000, st)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("method,info", [("voxel", {"voxel_size": 0.01}), ("random", {"downsample_ratio": 0.5}),
                                         ("fps", {"downsample_ratio": 0.1})])
def test_refine_with_downsampling(device, method, info):
    """FeaturePredictor's downsample branch (feature_predictor.py:159-196): the backbone runs on the downsampled
    cloud and its features are mapped back; reproducible for a fixed seed (to the conv's float-atomic order),
    finite, full-size output."""
    from splatformer_amd.feature_predictor import FeaturePredictor
    from splatformer_amd.scenes import make_scene, to_device
    torch.manual_seed(0)
    model = FeaturePredictor(sh_degree=1, zeroinit=False, additional_info=dict(downsample=method, **info))
    model = model.eval().to(device)
    scene = to_device(make_scene(3000, 1, seed=9), device)
    outs = []
    for _ in range(2):
        torch.manual_seed(1)
        outs.append(model.refine_packed(scene, perms=[[0, 1, 2, 3]] * 5).clone())
    assert outs[0].shape[0] == 3000 and torch.isfinite(outs[0]).all()
    assert float((outs[0] - outs[1]).norm() / outs[1].norm()) < 1e-5


def test_empty_samples_rejected(device):
    """A ratio with int(N * ratio) == 0 keeps no point: rejected on the host (the 1-NN map-back would index an
    empty tensor)."""
    pts = torch.rand(100, 3, device=device)
    feat = torch.rand(100, 4, device=device)
    grid = (pts * 384).int()
    with pytest.raises(ValueError):
        ds.fps_knn_downsample(pts, feat, grid, 0.001)
    with pytest.raises(ValueError):
        ds.random_downsample(pts, feat, grid, 0.001)
    with pytest.raises(ValueError):
        ds.nn1(pts, pts[:0])
