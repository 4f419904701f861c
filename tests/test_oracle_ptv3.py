"""CPU tests of the PTv3/FeaturePredictor oracle: golden vectors from the reference's
feature_predictor.py (tests/golden/feature_predictor.npz) and serialization KATs."""
import os

import numpy as np
import pytest
import torch

from oracle import ptv3_ref, serialize_ref

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "feature_predictor.npz")


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD))


def test_batchify_matches_reference(gold):
    s = {k[3:]: torch.from_numpy(v) for k, v in gold.items() if k.startswith("in_")}
    d = ptv3_ref.batchify(s)
    np.testing.assert_array_equal(d["feat"].numpy(), gold["bb_feat"])
    np.testing.assert_array_equal(d["coord"].numpy(), gold["bb_coord"])
    np.testing.assert_array_equal(d["grid_coord"].numpy(), gold["bb_grid_coord"])
    np.testing.assert_array_equal(d["offset"].numpy(), gold["bb_offset"])
    np.testing.assert_allclose(d["grid_size"].numpy(), gold["bb_grid_size"])


def test_heads_match_reference(gold):
    s = {k[3:]: torch.from_numpy(v) for k, v in gold.items() if k.startswith("in_")}
    sd = {"features_outputhead." + k[5:]: torch.from_numpy(v) for k, v in gold.items() if k.startswith("head.")}
    y = torch.from_numpy(gold["bb_out"])
    feat = torch.from_numpy(gold["bb_feat"])
    out = ptv3_ref.heads_forward(sd, y, feat, s)
    for k in ["means", "scales", "opacities", "quats", "features_dc", "features_rest"]:
        np.testing.assert_allclose(out[k].numpy(), gold["out_" + k], rtol=1e-6, atol=1e-6)


def test_product_module_state_dict_keys(gold):
    """The MI355X FeaturePredictor exposes the reference's head parameter names and shapes."""
    from splatformer_amd.feature_predictor import FeaturePredictor
    m = FeaturePredictor(sh_degree=1, zeroinit=False)
    hs = m.features_outputhead.state_dict()
    for k, v in gold.items():
        if k.startswith("head."):
            assert k[5:] in hs and tuple(hs[k[5:]].shape) == v.shape
    keys = m.state_dict().keys()
    for k in ["backbone.backbone.embedding.0.weight", "backbone.backbone.embedding.1.running_var",
              "backbone.backbone.enc.enc0.block0.cpe.0.weight", "backbone.backbone.enc.enc1.down.proj.weight",
              "backbone.backbone.enc.enc1.down.norm.0.running_mean", "backbone.backbone.enc.enc3.block5.mlp.0.fc2.bias",
              "backbone.backbone.dec.dec0.up.proj_skip.1.weight", "backbone.backbone.dec.dec0.block1.attn.qkv.weight",
              "backbone.backbone.dec.dec3.up.proj.0.weight"]:
        assert k in keys, k
    assert tuple(m.state_dict()["backbone.backbone.enc.enc0.block0.cpe.0.weight"].shape) == (64, 3, 3, 3, 64)
    n_params = sum(p.numel() for p in m.parameters())
    assert 40e6 < n_params < 60e6  # ~47.9 M parameters


def test_z_order_unit_vectors():
    g = np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1], [3, 0, 0], [256, 0, 0]])
    c = serialize_ref.z_order_encode(g, 9)
    assert c.tolist() == [0b100, 0b010, 0b001, 0b100100, 1 << 26]


@pytest.mark.parametrize("depth", [1, 2, 3])
def test_hilbert_is_a_face_adjacent_path(depth):
    side = 1 << depth
    ax = np.arange(side)
    g = np.stack(np.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(-1, 3)
    c = serialize_ref.hilbert_encode(g, depth)
    assert sorted(c.tolist()) == list(range(side ** 3))  # bijection
    path = g[np.argsort(c)]
    steps = np.abs(np.diff(path, axis=0)).sum(1)
    assert (steps == 1).all()  # consecutive codes are face-adjacent cells


def test_serialization_batch_bits_and_inverse():
    rng = np.random.default_rng(0)
    g = rng.integers(0, 384, size=(500, 3))
    b = np.repeat(np.arange(2), 250)
    code, order, inverse, depth = serialize_ref.serialization(g, b, perm=[2, 0, 3, 1])
    assert depth == 9
    assert (code[:, 250:] >> 27 == 1).all() and (code[:, :250] >> 27 == 0).all()
    for r in range(4):
        assert (order[r][inverse[r]] == np.arange(500)).all()
        assert (np.diff(code[r][order[r]]) >= 0).all()


def test_subm_neighbors_oracle():
    grid = torch.tensor([[1, 1, 1], [2, 1, 1], [1, 1, 2], [1, 1, 1]])
    nbr = ptv3_ref.subm_neighbors(grid, torch.zeros(4, dtype=torch.int64))
    assert nbr[0, 13] == 0 and nbr[3, 13] == 0       # duplicate voxel -> lowest index
    assert nbr[0, 22] == 1 and nbr[1, 4] == 0        # +x / -x
    assert nbr[0, 14] == 2 and nbr[2, 12] == 0       # +z / -z
    assert (nbr >= -1).all()
