"""The oracle's PTv3 backbone math vs code the reference itself holds (tests/golden/make_golden_backbone.py):

* visualize.py:129-243 (the SerializedAttention hook: pad / order / inverse, reshape / permute, scale,
  softmax, attn @ v, per-head inverse gather) -> oracle/ptv3_ref.py serialized_attention_heads;
* calflops.py:37-82 (the Block hook: cpe + shortcut, pre-norm norm1, attn, drop_path + shortcut, norm2)
  -> oracle/ptv3_ref.py block (its norm1 / norm2 outputs).
Bit-exact on the machine the goldens were made on; 1e-6 relative elsewhere (torch's CPU kernels may round
differently on another vector ISA)."""
import os

import numpy as np
import pytest
import torch

from oracle import ptv3_ref

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "backbone_pins.npz")


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD))


def _close(got, exp, what):
    got, exp = np.asarray(got, np.float64), np.asarray(exp, np.float64)
    assert got.shape == exp.shape, what
    err = np.abs(got - exp).max() / max(np.abs(exp).max(), 1e-30)
    assert err <= 1e-6, f"{what}: max rel err {err:.3e}"


def test_attention_matches_visualize_hook(gold):
    C, H, oi = int(gold["attn_C"]), int(gold["attn_H"]), int(gold["attn_order_index"])
    sd = {"a.qkv.weight": torch.from_numpy(gold["attn_qkv_w"]), "a.qkv.bias": torch.from_numpy(gold["attn_qkv_b"])}
    point = ptv3_ref.Point(offset=torch.from_numpy(gold["attn_offset"]),
                           serialized_order=torch.from_numpy(gold["attn_order"]),
                           serialized_inverse=torch.from_numpy(gold["attn_inverse"]))
    feat = torch.from_numpy(gold["attn_feat"])
    out = ptv3_ref.serialized_attention_heads(sd, "a", point, C, H, 128, oi, feat)
    d = C // H
    heads = gold["attn_heads"]
    assert heads.shape == (H, feat.shape[0], d)
    for i in range(H):
        _close(out[:, i * d:(i + 1) * d].numpy(), heads[i], f"head {i}")
    qkv = ptv3_ref.linear(feat, sd, "a.qkv")
    _close(qkv[:, 2 * C:2 * C + d].numpy(), gold["attn_value0"], "v (head 0)")


def test_block_order_matches_calflops_hook(gold):
    C, H, oi = int(gold["blk_C"]), int(gold["blk_H"]), int(gold["blk_order_index"])
    sd = {k[len("blk_sd."):]: torch.from_numpy(v) for k, v in gold.items() if k.startswith("blk_sd.")}
    grid = torch.from_numpy(gold["blk_grid"])
    offset = torch.from_numpy(gold["blk_offset"])
    point = ptv3_ref.Point(feat=torch.from_numpy(gold["blk_feat"]), offset=offset, grid_coord=grid,
                           serialized_order=torch.from_numpy(gold["blk_order"]),
                           serialized_inverse=torch.from_numpy(gold["blk_inverse"]))
    point.batch = ptv3_ref.offset2batch(offset)
    point.nbr = ptv3_ref.subm_neighbors(grid, point.batch)
    trace = {}
    ptv3_ref.block(sd, "blk", point, C, H, ptv3_ref.PTv3Config(), oi, trace=trace)
    _close(trace["h1"].numpy(), gold["blk_h1"], "norm1 output (attention input)")
    _close(trace["h2"].numpy(), gold["blk_h2"], "norm2 output (MLP input)")
