"""The SubMConv3d tap convention.

Convention (stated in DESIGN.md §7 and INTEGRATION.md): the spconv weight `weight[o, i, j, k, c]` ([Cout, 3, 3, 3,
Cin], spconv 2.x) multiplies input channel c of the active site at p + (i-1, j-1, k-1), where the three spatial
axes are the columns of Pointcept's sparse indices `[batch, x, y, z]` = grid_coord's (x, y, z) (Point.sparsify
[UPSTREAM], the input the reference's PointSequential hands to spconv: pointtransformer_v3.py:59-64).  That is
spconv's documented contract: a submanifold conv equals the dense cross-correlation (torch conv3d, padding 1)
evaluated at the active sites, with absent sites contributing zero.

On a fully occupied box every site is active, so SubM == conv3d(dense, weight.permute(0, 4, 1, 2, 3), padding=1)
everywhere -- with random (asymmetric) weights this fixes the tap order: a p - delta (flipped) kernel, a swapped
axis order or a transposed [Cin, Cout] read all fail it.  A real `train-on-objaverse.pth` (train.py:405-407) then
either loads correctly or differs from spconv in this one documented place.  spconv itself is absent here, so
the equality to spconv is parity unpinned; the equality to conv3d is what this pins.
"""
import pytest
import torch
import torch.nn.functional as F

from oracle import ptv3_ref


def _box(dx, dy, dz, origin=(3, 5, 7)):
    g = torch.stack(torch.meshgrid(torch.arange(dx), torch.arange(dy), torch.arange(dz), indexing="ij"), -1)
    return (g.reshape(-1, 3) + torch.tensor(origin)).int()


def _dense_ref(grid, x, weight, bias, origin, shape):
    """conv3d over the dense box (zero padding = absent neighbours), read back at the active sites."""
    cin = x.shape[1]
    vol = torch.zeros(1, cin, *shape, dtype=x.dtype)
    loc = (grid - torch.tensor(origin)).long()
    vol[0, :, loc[:, 0], loc[:, 1], loc[:, 2]] = x.T
    y = F.conv3d(vol, weight.permute(0, 4, 1, 2, 3).contiguous(), bias, padding=1)
    return y[0, :, loc[:, 0], loc[:, 1], loc[:, 2]].T


def _case(seed=0, shape=(5, 6, 7), cin=8, cout=12, dtype=torch.float64):
    g = torch.Generator().manual_seed(seed)
    origin = (3, 5, 7)
    grid = _box(*shape, origin=origin)
    perm = torch.randperm(grid.shape[0], generator=g)  # point order is irrelevant to the result
    grid = grid[perm].contiguous()
    x = torch.randn(grid.shape[0], cin, generator=g, dtype=dtype)
    w = torch.randn(cout, 3, 3, 3, cin, generator=g, dtype=dtype)
    b = torch.randn(cout, generator=g, dtype=dtype)
    return grid, x, w, b, origin, shape


def test_oracle_subm_equals_dense_conv3d_on_full_box():
    grid, x, w, b, origin, shape = _case()
    nbr = ptv3_ref.subm_neighbors(grid, torch.zeros(grid.shape[0], dtype=torch.int64))
    got = ptv3_ref.subm_conv(x, nbr, w, b)
    ref = _dense_ref(grid, x, w, b, origin, shape)
    assert torch.allclose(got, ref, rtol=1e-10, atol=1e-10)


def test_single_tap_direction():
    """One non-zero tap, weight[:, 2, 1, 1, :] (delta = (+1, 0, 0) on x): site p reads site p + x-hat."""
    grid = _box(4, 3, 3)
    n = grid.shape[0]
    x = torch.arange(n, dtype=torch.float64)[:, None]
    w = torch.zeros(1, 3, 3, 3, 1, dtype=torch.float64)
    w[0, 2, 1, 1, 0] = 1.0
    nbr = ptv3_ref.subm_neighbors(grid, torch.zeros(n, dtype=torch.int64))
    got = ptv3_ref.subm_conv(x, nbr, w, torch.zeros(1, dtype=torch.float64))[:, 0]
    key = {tuple(p.tolist()): i for i, p in enumerate(grid)}
    for i, p in enumerate(grid.tolist()):
        j = key.get((p[0] + 1, p[1], p[2]))
        assert got[i] == (float(j) if j is not None else 0.0)


@pytest.mark.gpu
def test_hip_subm_equals_dense_conv3d_on_full_box(device):
    from splatformer_amd import ptv3_ops as ops
    for cin, cout in ((8, 12), (64, 64), (96, 96)):  # exact-fp32 (K < 64) and fp16x2 launches
        grid, x, w, b, origin, shape = _case(seed=cin, cin=cin, cout=cout, dtype=torch.float32)
        ref = _dense_ref(grid, x.double(), w.double(), b.double(), origin, shape)
        smap = ops.subm_neighbors(grid.to(device), None)
        for partials in (False, True) if cin == cout and cout in ops.PAIRS_LN_CHANNELS else (False,):
            t = ops.subm_conv(x.to(device), smap, w.reshape(cout, -1).to(device), b.to(device), partials=partials)
            got = (t.total() if partials else t).cpu().double()
            err = float((got - ref).norm() / ref.norm())
            assert err < 2e-6, (cin, cout, partials, err)
