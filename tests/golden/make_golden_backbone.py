"""Capture golden vectors that pin the oracle's PTv3 backbone math with code the reference itself holds
(run in the build container only; /root/reference does not exist on the GPU box).

Pointcept is absent from the reference, but two of the reference's own scripts restate parts of it:

1. `visualize.py` `Model.register_get_feature_hook` (:129-243): a forward hook on SerializedAttention that
   recomputes the non-flash attention -- pad / order / inverse, qkv reshape / permute, q * scale @ k^T,
   softmax, attn @ v, and the per-head inverse gather.  Its source is extracted from the file (ast) and run
   on a stand-in attention module whose pieces are the oracle's (qkv Linear with seeded weights, Pointcept's
   get_padding_and_inverse as the oracle restates it; token merging at its "base" identity: process_merging
   returns q, k, v, size = 1, process_unreduction returns its input).  Recorded: per-head attention outputs
   (`ori_attn_feats`) and head-0 values for every point.
2. `calflops.py` `register_hooks` (:37-82): a forward hook on Block that replays the Block's order of
   operations (cpe + shortcut, pre-norm norm1, attn, drop_path + shortcut, norm2).  Run with the oracle's
   primitives as the Block's submodules and a recording FlopCountAnalysis stub (fvcore is absent): the norm1
   output handed to the attention FLOP count and the norm2 output handed to the MLP FLOP count are recorded.

3. The two real point clouds the reference ships (test/scene0140_01.bin, test/scene0451_01.bin; layout per
   test/js/scene.js:121-123 -- float32 positions [N,3], float32 normals [N,3], uint8 colours [N,3]): their
   positions and colours are stored as fixtures (data the reference's own test directory holds) for the
   serialization / neighbour-map / pooling parity tests on real geometry.

Outputs: tests/golden/backbone_pins.npz, tests/golden/real_clouds.npz.
"""
from __future__ import annotations

import ast
import os
import sys
from collections import defaultdict

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(OUT))
sys.path.insert(0, ROOT)

from oracle import ptv3_ref  # noqa: E402


def extract(path, qualname, namespace):
    """Exec the source of one function of a reference file (Class.method or function) in `namespace`."""
    tree = ast.parse(open(path).read())
    parts = qualname.split(".")
    body = tree.body
    node = None
    for part in parts:
        node = next(n for n in body if isinstance(n, (ast.FunctionDef, ast.ClassDef)) and n.name == part)
        body = node.body
    src = ast.unparse(node)
    exec(compile(src, f"{path}:{qualname}", "exec"), namespace)
    return namespace[parts[-1]]


class RPoint(dict):
    """addict-style Point whose copy() keeps attribute access (Pointcept Point.copy)."""
    __getattr__ = dict.__getitem__

    def __setattr__(self, k, v):
        self[k] = v

    def copy(self):
        return RPoint(self)


def scene_point(n, seed, C):
    from splatformer_amd.scenes import make_scene
    s = make_scene(n, 1, seed=seed, unique_voxels=True)
    data = ptv3_ref.batchify(s)
    p = ptv3_ref.Point(coord=data["coord"], grid_coord=data["grid_coord"], offset=data["offset"])
    p.batch = ptv3_ref.offset2batch(p.offset)
    ptv3_ref.serialize(p, [0, 1, 2, 3])
    g = torch.Generator().manual_seed(seed + 1)
    p.feat = torch.randn(p.coord.shape[0], C, generator=g)
    return p


def attention_pin(rec):
    N_SEED, C, H, order_index = 5, 64, 4, 1
    p = scene_point(2000, N_SEED, C)
    K = min(int(ptv3_ref.offset2bincount(p.offset).min()), 128)
    g = torch.Generator().manual_seed(77)
    qkv = torch.nn.Linear(C, 3 * C)
    with torch.no_grad():
        qkv.weight.copy_(torch.randn(3 * C, C, generator=g) / C ** 0.5)
        qkv.bias.copy_(torch.randn(3 * C, generator=g) * 0.1)

    class StandInAttention(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.qkv = qkv
            self.num_heads, self.patch_size, self.channels = H, K, C
            self.scale = (C // H) ** -0.5
            self.order_index = order_index
            self.softmax = torch.nn.Softmax(dim=-1)
            self.attn_drop = torch.nn.Dropout(0.0)
            self.additional_info = {"tome": "base", "tome_attention": True}

        def get_padding_and_inverse(self, point):
            pad, unpad = ptv3_ref.get_padding_and_inverse(point.offset, self.patch_size)
            return pad, unpad, None

        def process_merging(self, q, k, v, order, inverse):  # "base": no merging
            ident = lambda x: x
            return q, k, v, torch.ones(1), ident, ident  # size 1 everywhere: attn + log(size) = attn

        def process_unreduction(self, x, unmerge):
            return unmerge(x)

        def forward(self, point):
            return point

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.attn = StandInAttention()

    ns = {"torch": torch, "np": np, "VALID_TOME_MODES": ["patch", "tome", "progressive", "pitome", "random_patch",
                                                           "base", "important_patch"]}
    hook_factory = extract(os.path.join(REF, "visualize.py"), "Model.register_get_feature_hook", ns)
    self_ = type("M", (), {})()
    self_.model = Net()
    cuda = torch.Tensor.cuda
    torch.Tensor.cuda = lambda t, *a, **k: t  # the hook moves two helper tensors to 'cuda'
    try:
        hooks, feats, names = hook_factory(self_, ["attn"])
        point = RPoint(coord=p.coord, feat=p.feat, offset=p.offset, serialized_order=p.serialized_order,
                       serialized_inverse=p.serialized_inverse)
        self_.model.attn(point)
    finally:
        torch.Tensor.cuda = cuda
    assert names == ["attn"] and len(feats) == 1
    f = feats[0]
    rec.update(attn_feat=p.feat.numpy(), attn_qkv_w=qkv.weight.detach().numpy(), attn_qkv_b=qkv.bias.detach().numpy(),
               attn_order=p.serialized_order.numpy(), attn_inverse=p.serialized_inverse.numpy(),
               attn_offset=p.offset.numpy(), attn_C=C, attn_H=H, attn_order_index=order_index, attn_K=K,
               attn_heads=np.stack([t.detach().numpy() for t in f["ori_attn_feats"]]),
               attn_value0=f["ori_value"].numpy())


def block_pin(rec):
    C, H, order_index = 64, 2, 0
    p = scene_point(1500, 9, C)
    p.nbr = ptv3_ref.subm_neighbors(p.grid_coord, p.batch)
    g = torch.Generator().manual_seed(31)
    pre = "blk"
    sd = {
        f"{pre}.cpe.0.weight": torch.randn(C, 3, 3, 3, C, generator=g) / (27 * C) ** 0.5,
        f"{pre}.cpe.0.bias": torch.randn(C, generator=g) * 0.1,
        f"{pre}.cpe.1.weight": torch.randn(C, C, generator=g) / C ** 0.5,
        f"{pre}.cpe.1.bias": torch.randn(C, generator=g) * 0.1,
        f"{pre}.cpe.2.weight": torch.rand(C, generator=g) + 0.5,
        f"{pre}.cpe.2.bias": torch.randn(C, generator=g) * 0.1,
        f"{pre}.norm1.0.weight": torch.rand(C, generator=g) + 0.5,
        f"{pre}.norm1.0.bias": torch.randn(C, generator=g) * 0.1,
        f"{pre}.attn.qkv.weight": torch.randn(3 * C, C, generator=g) / C ** 0.5,
        f"{pre}.attn.qkv.bias": torch.randn(3 * C, generator=g) * 0.1,
        f"{pre}.attn.proj.weight": torch.randn(C, C, generator=g) / C ** 0.5,
        f"{pre}.attn.proj.bias": torch.randn(C, generator=g) * 0.1,
        f"{pre}.norm2.0.weight": torch.rand(C, generator=g) + 0.5,
        f"{pre}.norm2.0.bias": torch.randn(C, generator=g) * 0.1,
        f"{pre}.mlp.0.fc1.weight": torch.randn(4 * C, C, generator=g) / C ** 0.5,
        f"{pre}.mlp.0.fc1.bias": torch.randn(4 * C, generator=g) * 0.1,
        f"{pre}.mlp.0.fc2.weight": torch.randn(C, 4 * C, generator=g) / (4 * C) ** 0.5,
        f"{pre}.mlp.0.fc2.bias": torch.randn(C, generator=g) * 0.1,
    }
    cfg = ptv3_ref.PTv3Config()

    def with_feat(point, feat):
        q = RPoint(point)
        q["feat"] = feat
        return q

    class Fn(torch.nn.Module):
        def __init__(self, fn):
            super().__init__()
            self.fn = fn

        def forward(self, point):
            return self.fn(point)

    def cpe(point):
        x = ptv3_ref.subm_conv(point.feat, p.nbr, sd[f"{pre}.cpe.0.weight"], sd[f"{pre}.cpe.0.bias"])
        x = ptv3_ref.linear(x, sd, f"{pre}.cpe.1")
        return with_feat(point, ptv3_ref.ln(x, sd, f"{pre}.cpe.2", cfg.ln_eps))

    def attn(point):
        opoint = ptv3_ref.Point(offset=p.offset, serialized_order=p.serialized_order,
                                serialized_inverse=p.serialized_inverse)
        return with_feat(point, ptv3_ref.serialized_attention(sd, f"{pre}.attn", opoint, C, H, cfg.patch_size,
                                                              order_index, point.feat))

    class StandInBlock(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.pre_norm = True
            self.cpe = Fn(cpe)
            self.norm1 = Fn(lambda pt: with_feat(pt, ptv3_ref.ln(pt.feat, sd, f"{pre}.norm1.0", cfg.ln_eps)))
            self.attn = Fn(attn)
            self.drop_path = Fn(lambda pt: pt)
            self.norm2 = Fn(lambda pt: with_feat(pt, ptv3_ref.ln(pt.feat, sd, f"{pre}.norm2.0", cfg.ln_eps)))
            self.mlp = Fn(lambda pt: pt)

        def forward(self, point):
            return point

    recorded = []

    class FlopCountAnalysis:  # fvcore stub: records the inputs the hook hands to the FLOP counter
        def __init__(self, module, inputs):
            recorded.append(inputs["feat"] if isinstance(inputs, dict) else inputs)

        def unsupported_ops_warnings(self, flag):
            return self

        def uncalled_modules_warnings(self, flag):
            return self

        def total(self):
            return 0.0

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.block0 = StandInBlock()

    ns = {"torch": torch, "defaultdict": defaultdict, "FlopCountAnalysis": FlopCountAnalysis,
          "Block": StandInBlock, "Point": RPoint}
    register_hooks = extract(os.path.join(REF, "calflops.py"), "register_hooks", ns)
    net = Net()
    hooks, gflops, names = register_hooks(net)
    assert names == ["block0"]
    point = RPoint(coord=p.coord, feat=p.feat, offset=p.offset, serialized_order=p.serialized_order,
                   serialized_inverse=p.serialized_inverse)
    net.block0(point)
    assert len(recorded) == 2
    rec.update(blk_feat=p.feat.numpy(), blk_grid=p.grid_coord.numpy(), blk_order=p.serialized_order.numpy(),
               blk_inverse=p.serialized_inverse.numpy(), blk_offset=p.offset.numpy(), blk_C=C, blk_H=H,
               blk_order_index=order_index, blk_h1=recorded[0].numpy(), blk_h2=recorded[1].numpy(),
               **{"blk_sd." + k: v.numpy() for k, v in sd.items()})


def real_clouds():
    out = {}
    for name, n in [("scene0140_01", 135046), ("scene0451_01", 107046)]:
        raw = open(os.path.join(REF, "test", name + ".bin"), "rb").read()
        assert len(raw) == 27 * n, name
        out[name + "_xyz"] = np.frombuffer(raw, np.float32, 3 * n, 0).reshape(n, 3).copy()
        out[name + "_rgb"] = np.frombuffer(raw, np.uint8, 3 * n, 24 * n).reshape(n, 3).copy()
    np.savez_compressed(os.path.join(OUT, "real_clouds.npz"), **out)


def main():
    torch.manual_seed(0)
    rec = {}
    attention_pin(rec)
    block_pin(rec)
    np.savez_compressed(os.path.join(OUT, "backbone_pins.npz"), **rec)
    real_clouds()
    print("wrote backbone_pins.npz, real_clouds.npz")


if __name__ == "__main__":
    main()
