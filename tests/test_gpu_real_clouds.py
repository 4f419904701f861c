"""Integer path on real geometry: the two ScanNet point clouds the reference ships (test/scene0140_01.bin,
135,046 points; test/scene0451_01.bin, 107,046 points; fixtures in tests/golden/real_clouds.npz, written by
tests/golden/make_golden_backbone.py).  Normalised as the dataset normalises Gaussian means
(MinMaxScaler, transform_utils.py:64-91) and voxelised at grid_resolution 384 (feature_predictor.py:156).

Bit-exact against the oracle / the reference's integer math at every stage of the ptv3_base encoder:
serialization codes / orders / inverses (4 orders), the 27-neighbour map and its offset-major pair lists,
and the sort-free pooling geometry (clusters, CSR pointers, pooled codes / orders / inverses / grid) through
the four poolings (strides 1, 2, 2, 2).  Plus a full HIP refine of one cloud (Gaussian attributes seeded,
colours from the file) vs the oracle (relative L2 of the residual <= 1e-5)."""
import os

import numpy as np
import pytest
import torch

from oracle import ptv3_ref, serialize_ref
from splatformer_amd import ptv3_ops as ops
from splatformer_amd.ptv3 import Point, SerializedPooling
from splatformer_amd.scenes import minmax_normalize

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "real_clouds.npz")
SCENES = ["scene0140_01", "scene0451_01"]


@pytest.fixture(scope="module")
def clouds():
    return dict(np.load(GOLD))


def _grid(clouds, name):
    xyz = torch.from_numpy(clouds[name + "_xyz"]).float()
    coord = minmax_normalize(xyz)
    return coord, torch.floor(coord * 384).int()


def _ref_pool(code_rows, stride, depth):
    """Pointcept SerializedPooling's integer half on logical rows (pointtransformer_v3.py:290-299)."""
    pd = (stride - 1).bit_length()
    if pd > depth:
        pd = 0
    code = code_rows >> 3 * pd
    _, cluster, counts = torch.unique(code[0], sorted=True, return_inverse=True, return_counts=True)
    indices = torch.sort(cluster, stable=True).indices
    ptr = torch.cat([counts.new_zeros(1), torch.cumsum(counts, 0)])
    head = indices[ptr[:-1]]
    code_h = code[:, head]
    order = torch.argsort(code_h, stable=True)
    inv = torch.zeros_like(order).scatter_(1, order, torch.arange(code_h.shape[1]).repeat(code.shape[0], 1))
    return pd, cluster, ptr, head, code_h, order, inv


@pytest.mark.parametrize("name", SCENES)
def test_real_cloud_integer_path(device, clouds, name):
    coord, grid = _grid(clouds, name)
    n = grid.shape[0]
    depth = int(grid.max()).bit_length()
    codes, order, inverse = ops.serialize(grid.to(device), None, depth, 3 * depth, ptv3_ref.ORDERS)
    c_ref, o_ref, i_ref, _ = serialize_ref.serialization(grid.numpy(), np.zeros(n, np.int64), ptv3_ref.ORDERS, None)
    assert np.array_equal(codes.cpu().numpy(), c_ref)
    assert np.array_equal(order.cpu().numpy(), o_ref)
    assert np.array_equal(inverse.cpu().numpy(), i_ref)
    perms = [[2, 0, 3, 1], [1, 3, 0, 2], [3, 2, 1, 0], [0, 2, 1, 3], [2, 3, 0, 1]]
    pt = Point(coord=coord.to(device), grid_coord=grid.to(device), offset=[n], codes_phys=codes, order_phys=order,
               inverse_phys=inverse, order_type=list(perms[0]), serialized_depth=depth, code_bits=3 * depth)
    code_l = torch.from_numpy(c_ref)[perms[0]]  # logical rows of the reference Point
    g_ref = grid.long()
    for s, stride in enumerate([None, 1, 2, 2, 2]):
        if stride is not None:
            new, sidx, idx_ptr, m = SerializedPooling(8, 8, stride=stride, norm_layer=torch.nn.BatchNorm1d,
                                                      act_layer=torch.nn.GELU).geometry(pt, perms[s])
            pd, cluster, ptr, head, code_h, order_r, inv_r = _ref_pool(code_l, stride, pt.serialized_depth)
            assert m == ptr.numel() - 1, f"stage {s}: {m} clusters vs {ptr.numel() - 1}"
            assert torch.equal(new.pooling_inverse.cpu().long(), cluster), f"stage {s}: clusters"
            assert torch.equal(idx_ptr.cpu().long(), ptr), f"stage {s}: idx_ptr"
            perm = torch.as_tensor(perms[s])
            rows = new.order_type
            assert torch.equal(new.codes_phys.cpu()[rows], code_h[perm]), f"stage {s}: codes"
            assert torch.equal(new.order_phys.cpu().long()[rows], order_r[perm]), f"stage {s}: orders"
            assert torch.equal(new.inverse_phys.cpu().long()[rows], inv_r[perm]), f"stage {s}: inverses"
            g_ref = g_ref[head] >> pd
            assert torch.equal(new.grid_coord.cpu().long(), g_ref), f"stage {s}: grid"
            code_l = code_h[perm]
            pt = new
        # neighbour map + offset-major pair lists of this stage
        smap = ops.subm_neighbors(pt.grid_coord, None)
        nbr_ref = ptv3_ref.subm_neighbors(pt.grid_coord.cpu(), torch.zeros(pt.grid_coord.shape[0], dtype=torch.long))
        assert torch.equal(smap.nbr.cpu().long(), nbr_ref), f"stage {s}: neighbour map"
        off = smap.pair_off
        pin, pout = smap.pair_in.cpu().long(), smap.pair_out.cpu().long()
        for k in range(27):
            rows_k = torch.nonzero(nbr_ref[:, k] >= 0).flatten() if k != 13 else torch.zeros(0, dtype=torch.long)
            assert torch.equal(pout[off[k]:off[k + 1]], rows_k), f"stage {s} offset {k}: pair outputs"
            assert torch.equal(pin[off[k]:off[k + 1]], nbr_ref[rows_k, k]), f"stage {s} offset {k}: pair inputs"


def test_real_cloud_refine(device, clouds):
    """FeaturePredictor on scene0451_01's geometry (107k points, ~zero duplicates removed): Gaussian attributes
    seeded, features_dc from the cloud's colours (RGB2SH)."""
    from splatformer_amd.feature_predictor import FeaturePredictor
    from splatformer_amd.scenes import to_device
    coord, _ = _grid(clouds, "scene0451_01")
    n = coord.shape[0]
    g = torch.Generator().manual_seed(451)
    rgb = torch.from_numpy(clouds["scene0451_01_rgb"]).float() / 255.0
    scene = {"means": coord.contiguous(),
             "scales": -5.5 + 0.5 * torch.randn(n, 3, generator=g),
             "quats": torch.randn(n, 4, generator=g),
             "opacities": 1.0 + 1.5 * torch.randn(n, 1, generator=g),
             "features_dc": ((rgb - 0.5) / 0.28209479177387814).contiguous(),
             "features_rest": 0.1 * torch.randn(n, 3, 3, generator=g)}
    torch.manual_seed(0)
    model = FeaturePredictor(sh_degree=1, zeroinit=False).eval()
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    model = model.to(device)
    with torch.no_grad():
        out = model([to_device(scene, device)], [0])[0]
    perms = model.backbone.backbone.last_perms
    ref, _ = ptv3_ref.feature_predictor_forward(sd, ptv3_ref.PTv3Config(), scene, perms)
    for k in ref:
        d = (out[k].cpu() - ref[k]).double()
        r = (ref[k] - scene[k]).double()
        err = float(d.norm() / r.norm().clamp_min(1e-30))
        assert err <= 1e-5, f"refined {k}: residual rel L2 {err:.3e}"
