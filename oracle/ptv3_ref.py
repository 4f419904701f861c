"""CPU restatement of the SplatFormer refiner: Pointcept PTv3 m1 (as assembled by
reference models/pointtransformer_v3.py) + FeaturePredictor heads
(reference models/feature_predictor.py:127-245).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Pointcept's modules live in the un-vendored hchautran/Pointcept submodule
(reference .gitmodules:1-3; empty in /root/reference).  Their semantics are
restated from the published PTv3 m1 code and the
in-tree restatements calflops.py:45-82 (Block order of operations) and
visualize.py:140-179 (non-flash attention math).  Functional form over a
state dict whose keys are the reference module's
(`backbone.embedding.0.weight`, `backbone.enc.enc0.block0.cpe.0.weight`, ...).
fp32 torch ops on the CPU; integer serialization via oracle.serialize_ref.
"""
from __future__ import annotations

import contextlib
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from . import serialize_ref

ORDERS = ("z", "z-trans", "hilbert", "hilbert-trans")


@dataclass
class PTv3Config:
    """ptv3_base.gin + PointTransformerV3Model defaults (pointtransformer_v3.py:83-161)."""
    in_channels: int = 23
    enc_depths: Sequence[int] = (2, 2, 2, 6, 2)
    enc_channels: Sequence[int] = (64, 96, 128, 256, 512)
    enc_num_head: Sequence[int] = (2, 4, 8, 16, 32)
    dec_depths: Sequence[int] = (2, 2, 2, 2)
    dec_channels: Sequence[int] = (96, 96, 128, 256)
    dec_num_head: Sequence[int] = (4, 4, 8, 16)
    stride: Sequence[int] = (1, 2, 2, 2)
    patch_size: int = 128
    enable_flash: bool = False  # Pointcept flash branch: fixed K = patch_size (1024 in the reference) windows
    mlp_ratio: int = 4
    bn_eps: float = 1e-3
    ln_eps: float = 1e-5

    @property
    def num_stages(self):
        return len(self.enc_depths)


# ---- autocast precision (reference train.py:240 `torch.cuda.amp.autocast(enabled=enable_amp)`,
# configs/train/default.gin:11) ------------------------------------------------------------------------------
# Under CUDA autocast the matmul-class ops (F.linear, the spconv SubM conv, the attention matmuls) take fp16
# operands, accumulate in fp32 and return fp16; LayerNorm / softmax run in fp32 on the (fp16) values they get;
# BatchNorm and GELU keep their fp16 input type.  The restatement stays an fp32 computation and rounds every
# value autocast would hold in fp16 to fp16 (`_h`); autograd through the roundings gives the fp16 gradients of
# those ops.  fp64 tensors pass through unchanged (the fp64 oracle is exact by construction).
AUTOCAST = False


def _h(t):
    return t.half().float() if (AUTOCAST and t is not None and t.dtype == torch.float32) else t


@contextlib.contextmanager
def autocast(enabled: bool = True):
    """Run the enclosed oracle calls in the reference's autocast precision."""
    global AUTOCAST
    prev, AUTOCAST = AUTOCAST, enabled
    try:
        yield
    finally:
        AUTOCAST = prev


def _lin(x, w, b):
    return _h(F.linear(_h(x), _h(w), _h(b)))


# ---- primitives -------------------------------------------------------------
def linear(x, sd, p):
    return _lin(x, sd[p + ".weight"], sd.get(p + ".bias"))


def bn(x, sd, p, eps, train=False):
    """Eval: running statistics.  Train (model.train(), train.py:236): batch statistics; the running
    statistics are updated on the state dict in place (momentum 0.01, pointtransformer_v3.py:252)."""
    if not train:
        return _h(F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"],
                               sd[p + ".bias"], False, 0.0, eps))
    return _h(F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"], sd[p + ".bias"],
                           True, 0.01, eps))


def ln(x, sd, p, eps):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], eps)


def gelu(x):
    return _h(F.gelu(x))


def subm_neighbors(grid: torch.Tensor, batch: torch.Tensor) -> torch.Tensor:
    """27-neighbour map (k = (dx+1)*9 + (dy+1)*3 + (dz+1)); duplicates resolve to the lowest index."""
    g = grid.numpy().astype(np.int64)
    b = batch.numpy().astype(np.int64)
    pack = lambda bb, x, y, z: (bb << 48) | ((x + 1) << 32) | ((y + 1) << 16) | (z + 1)
    keys = pack(b, g[:, 0], g[:, 1], g[:, 2])
    uniq, first = np.unique(keys, return_index=True)  # first occurrence == lowest index
    nbr = np.full((g.shape[0], 27), -1, dtype=np.int64)
    for k in range(27):
        dx, dy, dz = k // 9 - 1, (k // 3) % 3 - 1, k % 3 - 1
        x, y, z = g[:, 0] + dx, g[:, 1] + dy, g[:, 2] + dz
        ok = (x >= 0) & (y >= 0) & (z >= 0)
        q = pack(b, x, y, z)
        pos = np.clip(np.searchsorted(uniq, q), 0, len(uniq) - 1)
        hit = ok & (uniq[pos] == q)
        nbr[hit, k] = first[pos[hit]]
    return torch.from_numpy(nbr)


def subm_conv(x, nbr, weight, bias):
    """spconv SubMConv3d (k=3): out_i = b + sum_k W[:,k,:] x_{nbr(i,k)}; weight [Cout,3,3,3,Cin]."""
    cout = weight.shape[0]
    W = weight.reshape(cout, 27, -1)
    out = torch.zeros(x.shape[0], cout, dtype=x.dtype)
    xz = torch.cat([_h(x), torch.zeros(1, x.shape[1], dtype=x.dtype)], 0)
    idx = torch.where(nbr < 0, torch.full_like(nbr, x.shape[0]), nbr)
    W = _h(W)
    for k in range(27):
        out = out + xz[idx[:, k]] @ W[:, k, :].T
    return _h(out + _h(bias))


# ---- Point ------------------------------------------------------------------
class Point(dict):
    __getattr__ = dict.__getitem__

    def __setattr__(self, k, v):
        self[k] = v


def offset2bincount(offset: torch.Tensor) -> torch.Tensor:
    return torch.diff(offset, prepend=torch.zeros(1, dtype=offset.dtype))


def offset2batch(offset: torch.Tensor) -> torch.Tensor:
    counts = offset2bincount(offset)
    return torch.repeat_interleave(torch.arange(len(counts)), counts)


def serialize(point: Point, perm):
    code, order, inverse, depth = serialize_ref.serialization(point.grid_coord.numpy(), point.batch.numpy(), ORDERS,
                                                              perm)
    point.serialized_code = torch.from_numpy(code)
    point.serialized_order = torch.from_numpy(order)
    point.serialized_inverse = torch.from_numpy(inverse)
    point.serialized_depth = depth


# ---- attention (SerializedAttention, enable_flash=False) -----------------------
def get_padding_and_inverse(offset: torch.Tensor, patch_size: int):
    bincount = offset2bincount(offset)
    bincount_pad = torch.div(bincount + patch_size - 1, patch_size, rounding_mode="trunc") * patch_size
    mask_pad = bincount > patch_size
    bincount_pad = ~mask_pad * bincount + mask_pad * bincount_pad
    _offset = F.pad(offset, (1, 0))
    _offset_pad = F.pad(torch.cumsum(bincount_pad, dim=0), (1, 0))
    pad = torch.arange(_offset_pad[-1])
    unpad = torch.arange(_offset[-1])
    for i in range(len(offset)):
        unpad[_offset[i]:_offset[i + 1]] += _offset_pad[i] - _offset[i]
        if bincount[i] != bincount_pad[i]:
            pad[_offset_pad[i + 1] - patch_size + (bincount[i] % patch_size):_offset_pad[i + 1]] = pad[
                _offset_pad[i + 1] - 2 * patch_size + (bincount[i] % patch_size):_offset_pad[i + 1] - patch_size]
        pad[_offset_pad[i]:_offset_pad[i + 1]] -= _offset_pad[i] - _offset[i]
    return pad, unpad


def cu_seqlens(offset: torch.Tensor, patch_size: int) -> torch.Tensor:
    """Pointcept get_padding_and_inverse's third output (the flash branch's window starts over the padded
    sequence + its end): arange(_offset_pad[i], _offset_pad[i+1], step=K) per batch."""
    bincount = offset2bincount(offset)
    bincount_pad = torch.div(bincount + patch_size - 1, patch_size, rounding_mode="trunc") * patch_size
    mask_pad = bincount > patch_size
    bincount_pad = ~mask_pad * bincount + mask_pad * bincount_pad
    _offset_pad = F.pad(torch.cumsum(bincount_pad, dim=0), (1, 0))
    cu = [torch.arange(_offset_pad[i], _offset_pad[i + 1], patch_size) for i in range(len(offset))]
    return F.pad(torch.cat(cu), (0, 1), value=int(_offset_pad[-1]))


def serialized_attention_flash(qkv, point: Point, C, H, K, order_index):
    """The enable_flash=True branch (reference pointtransformer_v3.py:121-123 -> Pointcept SerializedAttention:
    patch K fixed, qkv[order] over the padded sequence, flash_attn_varlen_qkvpacked_func over cu_seqlens windows,
    feat[inverse]).  Pointcept casts qkv to fp16 for flash-attn; this restatement keeps fp32 (fp64 when qkv is).
    Parity of the varlen window cut against a flash-attn run is unpinned (Pointcept / flash-attn are absent)."""
    pad, unpad = get_padding_and_inverse(point.offset, K)
    cu = cu_seqlens(point.offset, K)
    order = point.serialized_order[order_index][pad]
    inverse = unpad[point.serialized_inverse[order_index]]
    q, k, v = qkv[order].reshape(-1, 3, H, C // H).unbind(dim=1)   # [Npad, H, d]
    scale = (C // H) ** -0.5
    out = torch.empty(q.shape[0], C, dtype=qkv.dtype)
    for s, e in zip(cu[:-1].tolist(), cu[1:].tolist()):
        a = torch.softmax(torch.einsum("qhd,khd->hqk", q[s:e] * scale, k[s:e]), dim=-1)
        out[s:e] = torch.einsum("hqk,khd->qhd", a, v[s:e]).reshape(e - s, C)
    return out[inverse]


def serialized_attention_heads(sd, p, point: Point, C, H, patch_size_max, order_index, feat, flash=False):
    """SerializedAttention up to (excluding) proj: the per-head softmax(q k^T d^-1/2) v of every point, heads
    concatenated along channels, in the original point order [N, C] (restated visualize.py:140-179; pinned by
    tests/golden/backbone_pins.npz captured from that hook).  flash=True: serialized_attention_flash."""
    if flash:
        return serialized_attention_flash(linear(feat, sd, p + ".qkv"), point, C, H, patch_size_max, order_index)
    K = min(int(offset2bincount(point.offset).min()), patch_size_max)
    key = ("pad", K)
    if key not in point:
        point[key] = get_padding_and_inverse(point.offset, K)
    pad, unpad = point[key]
    order = point.serialized_order[order_index][pad]
    inverse = unpad[point.serialized_inverse[order_index]]
    qkv = linear(feat, sd, p + ".qkv")[order]
    q, k, v = qkv.reshape(-1, K, 3, H, C // H).permute(2, 0, 3, 1, 4).unbind(dim=0)
    scale = (C // H) ** -0.5
    attn = _h(_h(q * scale) @ k.transpose(-2, -1))
    attn = torch.softmax(attn, dim=-1)
    out = _h(_h(attn) @ v).transpose(1, 2).reshape(-1, C)
    return out[inverse]


def serialized_attention(sd, p, point: Point, C, H, patch_size_max, order_index, feat, flash=False):
    out = serialized_attention_heads(sd, p, point, C, H, patch_size_max, order_index, feat, flash)
    return linear(out, sd, p + ".proj")


# ---- Block ------------------------------------------------------------------
def block(sd, p, point: Point, C, H, cfg: PTv3Config, order_index, conv_in=None, masks=None, trace=None):
    """Block.forward (pre_norm=True; calflops.py:45-82, pinned by tests/golden/backbone_pins.npz).  DropPath
    (train): `masks[p + '.attn' / '.mlp']` = the per-point keep/(1-p) multipliers timm's DropPath draws
    (identity in eval / when absent).  `trace` (a dict) receives the norm1 / norm2 outputs (attention and MLP
    inputs) as "h1" / "h2"."""
    masks = masks or {}
    shortcut = point.feat
    x = subm_conv(point.feat if conv_in is None else conv_in, point.nbr, sd[p + ".cpe.0.weight"],
                  sd[p + ".cpe.0.bias"])
    x = linear(x, sd, p + ".cpe.1")
    x = ln(x, sd, p + ".cpe.2", cfg.ln_eps)
    feat = shortcut + x
    shortcut = feat
    h = ln(feat, sd, p + ".norm1.0", cfg.ln_eps)
    if trace is not None:
        trace["h1"] = h
    h = serialized_attention(sd, p + ".attn", point, C, H, cfg.patch_size, order_index, h, cfg.enable_flash)
    if masks.get(p + ".attn") is not None:
        h = h * masks[p + ".attn"][:, None]
    feat = shortcut + h
    shortcut = feat
    h = ln(feat, sd, p + ".norm2.0", cfg.ln_eps)
    if trace is not None:
        trace["h2"] = h
    h = linear(gelu(linear(h, sd, p + ".mlp.0.fc1")), sd, p + ".mlp.0.fc2")
    if masks.get(p + ".mlp") is not None:
        h = h * masks[p + ".mlp"][:, None]
    point.feat = shortcut + h
    return point


# ---- pooling / unpooling ------------------------------------------------------
def serialized_pooling(sd, p, point: Point, stride, cfg: PTv3Config, perm, train=False):
    pooling_depth = (math.ceil(stride) - 1).bit_length()
    if pooling_depth > point.serialized_depth:
        pooling_depth = 0
    code = point.serialized_code >> pooling_depth * 3
    code_, cluster, counts = torch.unique(code[0], sorted=True, return_inverse=True, return_counts=True)
    indices = torch.sort(cluster, stable=True).indices
    idx_ptr = torch.cat([counts.new_zeros(1), torch.cumsum(counts, dim=0)])
    head_indices = indices[idx_ptr[:-1]]
    code = code[:, head_indices]
    order = torch.argsort(code, stable=True)
    inverse = torch.zeros_like(order).scatter_(1, order, torch.arange(code.shape[1]).repeat(code.shape[0], 1))
    if perm is not None:
        perm = torch.as_tensor(perm)
        code, order, inverse = code[perm], order[perm], inverse[perm]
    proj = linear(point.feat, sd, p + ".proj")[indices]
    seg = torch.repeat_interleave(torch.arange(len(counts)), counts)
    feat = torch.full((len(counts), proj.shape[1]), -float("inf")).scatter_reduce(
        0, seg[:, None].expand_as(proj), proj, reduce="amax", include_self=True)
    csum = torch.zeros(len(counts), 3).index_add_(0, seg, point.coord[indices])
    coord = csum / counts[:, None].to(torch.float32)
    new = Point(feat=feat, coord=coord, grid_coord=point.grid_coord[head_indices] >> pooling_depth,
                serialized_code=code, serialized_order=order, serialized_inverse=inverse,
                serialized_depth=point.serialized_depth - pooling_depth, batch=point.batch[head_indices],
                pooling_inverse=cluster, pooling_parent=point)
    new.offset = torch.cumsum(torch.bincount(new.batch), 0)
    new.feat = gelu(bn(new.feat, sd, p + ".norm.0", cfg.bn_eps, train))
    return new


def serialized_unpooling(sd, p, point: Point, cfg: PTv3Config, train=False):
    parent = point.pooling_parent
    inverse = point.pooling_inverse
    coarse = gelu(bn(linear(point.feat, sd, p + ".proj.0"), sd, p + ".proj.1", cfg.bn_eps, train))
    skip = gelu(bn(linear(parent.feat, sd, p + ".proj_skip.0"), sd, p + ".proj_skip.1", cfg.bn_eps, train))
    parent.feat = _h(skip + coarse[inverse])  # (two fp16 tensors under autocast)
    parent.stale_conv_feat = skip  # sparse_conv_feat is not refreshed by SerializedUnpooling
    return parent


# ---- whole backbone -----------------------------------------------------------
def ptv3_forward(sd: Dict[str, torch.Tensor], cfg: PTv3Config, data: Dict[str, torch.Tensor],
                 perms: List[Sequence[int]], prefix: str = "backbone.", train: bool = False,
                 masks: Optional[Dict[str, torch.Tensor]] = None) -> Point:
    """PointTransformerV3.forward (pointtransformer_v3.py:378-392); `perms` = the 5 randperm(4) draws.
    train=True: batch-statistics BatchNorm + the DropPath `masks` (keys '<enc.enc0.block1>.attn' / '.mlp')."""
    sd = {k[len(prefix):]: v for k, v in sd.items() if k.startswith(prefix)}
    point = Point(coord=data["coord"], grid_coord=data["grid_coord"], offset=data["offset"], feat=data["feat"])
    point.batch = offset2batch(point.offset)
    serialize(point, perms[0])
    point.nbr = subm_neighbors(point.grid_coord, point.batch)
    # embedding: Linear -> BN -> GELU
    point.feat = gelu(bn(linear(point.feat, sd, "embedding.0"), sd, "embedding.1", cfg.bn_eps, train))
    pi = 1
    for s in range(cfg.num_stages):
        if s > 0:
            point = serialized_pooling(sd, f"enc.enc{s}.down", point, cfg.stride[s - 1], cfg, perms[pi], train)
            pi += 1
            point.nbr = subm_neighbors(point.grid_coord, point.batch)
        for i in range(cfg.enc_depths[s]):
            point = block(sd, f"enc.enc{s}.block{i}", point, cfg.enc_channels[s], cfg.enc_num_head[s], cfg, i % 4,
                          masks=masks)
    for s in reversed(range(cfg.num_stages - 1)):
        point = serialized_unpooling(sd, f"dec.dec{s}.up", point, cfg, train)
        for i in range(cfg.dec_depths[s]):
            conv_in = point.pop("stale_conv_feat") if i == 0 else None
            point = block(sd, f"dec.dec{s}.block{i}", point, cfg.dec_channels[s], cfg.dec_num_head[s], cfg, i % 4,
                          conv_in=conv_in, masks=masks)
    return point


# ---- FeaturePredictor (feature_predictor.py:127-245) ----------------------------
INPUT_FEATURES = ["means", "scales", "opacities", "quats", "features_dc", "features_rest"]
FEATURE2CHANNEL = {"means": 3, "features_dc": 3, "features_rest": 3, "opacities": 1, "scales": 3, "quats": 4}


def batchify(gs: Dict[str, torch.Tensor], grid_resolution: int = 384):
    feat = torch.cat([gs[k] if k != "features_rest" else gs[k].reshape(gs[k].shape[0], -1)
                      for k in INPUT_FEATURES if k in gs], dim=1)
    coord = gs["means"]
    return dict(coord=coord, grid_size=torch.ones(3) * 1.0 / grid_resolution,
                offset=torch.tensor([coord.shape[0]]), feat=feat,
                # feature_predictor.py:156 on the fp32 means (an fp64 check run keeps the fp32 voxel geometry)
                grid_coord=torch.floor(coord.float() * grid_resolution).int())


def heads_forward(sd, y: torch.Tensor, feat: torch.Tensor, in_gs: Dict[str, torch.Tensor], sh_degree: int = 1,
                  nlayer: int = 4, prefix: str = "features_outputhead.", relu_masks=None):
    """cat(y, feat) -> per-feature MLP(ReLU) -> tanh(means) -> residual add.

    relu_masks (test replay only): {feature: [active mask of hidden layer li]} -- each ReLU then keeps exactly
    the given active set (z * mask), so a gradient comparison is not decided by ReLU inputs that lie within
    rounding of 0 (whose sign differs between two fp32 evaluation orders)."""
    h0 = torch.cat([y, feat], 1)
    out = {}
    for f in INPUT_FEATURES:
        if f == "features_rest" and sh_degree == 0:
            continue
        h = h0
        for li in range(nlayer - 1):
            z = _lin(h, sd[f"{prefix}{f}.{2 * li}.weight"], sd[f"{prefix}{f}.{2 * li}.bias"])
            h = torch.relu(z) if relu_masks is None else z * relu_masks[f][li].to(z.dtype)
        o = _lin(h, sd[f"{prefix}{f}.{2 * (nlayer - 1)}.weight"], sd[f"{prefix}{f}.{2 * (nlayer - 1)}.bias"])
        if f == "means":
            o = _h(torch.tanh(o))
        if f == "features_rest":
            o = o.view(o.shape[0], -1, 3)
        out[f] = in_gs[f] + o
    return out


def feature_predictor_forward(sd, cfg: PTv3Config, gs: Dict[str, torch.Tensor], perms, sh_degree=1,
                              grid_resolution=384, train=False, masks=None, relu_masks=None):
    data = batchify(gs, grid_resolution)
    point = ptv3_forward(sd, cfg, data, perms, prefix="backbone.backbone.", train=train, masks=masks)
    return heads_forward(sd, point.feat, data["feat"], gs, sh_degree, relu_masks=relu_masks), point
