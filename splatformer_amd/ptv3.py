"""PointTransformerV3Model on MI355X: module tree of the reference, HIP forward.

Mirrors reference models/pointtransformer_v3.py:81-392 (the SplatFormer
assembly of Pointcept's PTv3 m1): same constructor arguments, same
submodule names and therefore the same state-dict keys
(`backbone.embedding.0.weight`, `backbone.enc.enc0.block0.cpe.0.weight`
([Cout,3,3,3,Cin] spconv layout), `...attn.qkv.weight`, `...mlp.0.fc1.weight`,
`backbone.dec.dec0.up.proj_skip.1.running_var`, ...), and
`forward(data_dict) -> Point` with `point["feat"]` the [N, dec_channels[0]]
feature the FeaturePredictor reads (feature_predictor.py:184-188).

The nn modules only hold parameters; forward runs entirely on libsfx HIP
kernels (serialization radix sort, 27-neighbour hash map, fp32-accurate MFMA
GEMMs with fused gather/BN/GELU/residual, windowed attention, pooling runs).
This module is the eval forward (the reference's eval path runs under
torch.no_grad(), train.py:81); the training forward/backward of the same
module tree (train-mode BN, DropPath, hand-written tape backward to the qkv
parameters) is `ptv3_train.py`, driven by `train.Trainer`.
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Sequence

import torch
import torch.nn as nn
from torch import Tensor

from . import _lib
from . import ptv3_ops as ops

ORDERS = ("z", "z-trans", "hilbert", "hilbert-trans")
# every pooling's cluster count from the stage-0 codes up front (default); SFX_POOL_COUNTS_UPFRONT=0 waits per pooling
POOL_COUNTS_UPFRONT = os.environ.get("SFX_POOL_COUNTS_UPFRONT", "1") != "0"


# the stage-0 SubM map is enqueued before the host waits for the grid depth (SFX_NBR_EARLY=0: after the serialization)
NBR_EARLY = os.environ.get("SFX_NBR_EARLY", "1") != "0"

class Point(dict):
    """addict-style dict (Pointcept `Point`) with attribute access."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


class SubMConv3d(nn.Module):
    """Parameter holder with spconv.SubMConv3d(C, C, kernel_size=3, bias=True) layout: weight [Cout,3,3,3,Cin]."""

    def __init__(self, in_channels, out_channels, kernel_size=3, bias=True, indice_key=None):
        super().__init__()
        assert kernel_size == 3
        self.in_channels, self.out_channels, self.indice_key = in_channels, out_channels, indice_key
        self.weight = nn.Parameter(torch.empty(out_channels, 3, 3, 3, in_channels))
        self.bias = nn.Parameter(torch.empty(out_channels)) if bias else None
        fan_in = in_channels * 27
        bound = 1.0 / math.sqrt(fan_in)
        nn.init.uniform_(self.weight, -math.sqrt(3.0) * bound, math.sqrt(3.0) * bound)
        if self.bias is not None:
            nn.init.uniform_(self.bias, -bound, bound)


class PointSequential(nn.Sequential):
    pass


class MLP(nn.Module):
    def __init__(self, in_channels, hidden_channels, out_channels):
        super().__init__()
        self.fc1 = nn.Linear(in_channels, hidden_channels)
        self.act = nn.GELU()
        self.fc2 = nn.Linear(hidden_channels, out_channels)
        self.drop = nn.Dropout(0.0)


class SerializedAttention(nn.Module):
    def __init__(self, channels, num_heads, patch_size, order_index=0, enable_flash=False):
        super().__init__()
        assert channels % num_heads == 0
        self.channels, self.num_heads = channels, num_heads
        # Pointcept's flash branch: fixed K = patch_size windows cut at cu_seqlens (a batch of n <= K points is
        # one n-key window) instead of K = min(min bincount, patch_size)
        self.enable_flash = enable_flash
        self.scale = (channels // num_heads) ** -0.5
        self.order_index = order_index
        self.patch_size_max = patch_size
        self.qkv = nn.Linear(channels, channels * 3, bias=True)
        self.proj = nn.Linear(channels, channels)
        self.attn_drop = nn.Dropout(0.0)
        self.proj_drop = nn.Dropout(0.0)
        self.softmax = nn.Softmax(dim=-1)


class Block(nn.Module):
    def __init__(self, channels, num_heads, patch_size=128, mlp_ratio=4.0, order_index=0, cpe_indice_key=None,
                 enable_flash=False):
        super().__init__()
        self.channels = channels
        self.pre_norm = True
        self.cpe = PointSequential(SubMConv3d(channels, channels, 3, True, cpe_indice_key),
                                   nn.Linear(channels, channels), nn.LayerNorm(channels))
        self.norm1 = PointSequential(nn.LayerNorm(channels))
        self.attn = SerializedAttention(channels, num_heads, patch_size, order_index, enable_flash)
        self.norm2 = PointSequential(nn.LayerNorm(channels))
        self.mlp = PointSequential(MLP(channels, int(channels * mlp_ratio), channels))
        self.drop_path = PointSequential(nn.Identity())  # DropPath has no parameters; rate in drop_prob
        self.drop_prob = 0.0

    def cpe_fused(self):
        """cpe = Linear(SubMConv3d(x)) folded into one sparse conv (exact in real arithmetic):
        W'_k = W_lin W_k, b' = W_lin b_conv + b_lin -- the per-point linear GEMM disappears.  Computed with
        the library GEMM, cached until one of the four tensors changes."""
        conv, lin = self.cpe[0], self.cpe[1]
        ts = (conv.weight, conv.bias, lin.weight, lin.bias)
        key = tuple((t.data_ptr(), t._version) for t in ts)
        cache = self.__dict__.get("_sfx_cpe")
        if cache is not None and cache[0] == key:
            return cache[1], cache[2]
        from .train_ops import transpose
        with torch.no_grad():
            C = self.channels
            wc = conv.weight.detach().reshape(C, -1)                   # [Cout, 27*Cin]
            wf = ops.linear(lin.weight.detach(), transpose(wc))        # W_lin @ Wc   [C, 27*Cin]
            bf = ops.linear(conv.bias.detach()[None].contiguous(), lin.weight.detach(), lin.bias.detach())[0]
        self.__dict__["_sfx_cpe"] = (key, wf.contiguous(), bf.contiguous())
        return wf, bf

    def cpe_packed(self):
        """cpe_fused() as the fused conv's fp16x2 fragment stream + inverse column scales (ops.subm_cpe_pack),
        cached until one of the four CPE tensors changes."""
        wf, bf = self.cpe_fused()
        key = self.__dict__["_sfx_cpe"][0]
        cache = self.__dict__.get("_sfx_cpe_pk")
        if cache is None or cache[0] != key:
            with torch.no_grad():
                wpk, winv = ops.subm_cpe_pack(wf)
            cache = (key, wpk, winv)
            self.__dict__["_sfx_cpe_pk"] = cache
        return cache[1], cache[2], bf

    def run(self, point: Point, conv_in: Optional[Tensor] = None, out: Optional[Tensor] = None) -> Point:
        """Block.forward (calflops.py:45-82): x += LN(Lin(SubMConv(x))); x += attn(LN1 x); x += MLP(LN2 x)."""
        x = point.feat
        C = self.channels
        ln_c = self.cpe[2]
        ln1 = self.norm1[0]
        xc = x if conv_in is None else conv_in
        fused = ops.subm_fused_ok(C, x.shape[0])
        if fused:
            # conv + LN_cpe + shortcut + norm1 in one launch, pair products summed on chip (csrc/subm_fused.hip);
            # the conv input's row exponents come from the previous Block's MLP epilogue when it wrote xc
            wpk, winv, bf = self.cpe_packed()
            re = point.get("feat_rowexp")
            x1, h = ops.subm_cpe_ln(xc, x, point.nbr, wpk, winv, bf, ln_c.weight, ln_c.bias, ln1.weight, ln1.bias,
                                    ln1.eps, rowexp=re[1] if re is not None and re[0] is xc else None)
        else:
            wf, bf = self.cpe_fused()
            # the conv's pair products go to per-pair rows that the LN kernel sums in a fixed order (no float
            # atomics, reproducible); SFX_SUBM_ATOMIC=1 restores the atomic accumulation
            t = ops.subm_conv(xc, point.nbr, wf, bf, partials=ops.subm_partials_ok(xc, point.nbr, C))
            if ops.cpe_ln_qkv_ok(t, C, self.attn.qkv.weight):
                # pair sums + LN_cpe + shortcut + norm1 + qkv in one launch: norm1's output never reaches HBM
                x1, qkv, q_amax = ops.cpe_ln_qkv(t, x, ln_c.weight, ln_c.bias, ln1.weight, ln1.bias, ln1.eps,
                                                 self.attn.qkv)
                h = None
            else:
                x1, h = ops.cpe_residual_ln(t, x, ln_c.weight, ln_c.bias, ln1.weight, ln1.bias, ln1.eps)
        # The GEMMs scale their fp16x2 operands per row themselves (no operand bounds needed); the qkv GEMM
        # publishes max |qkv| for the attention's fp16x2 q / k / v terms (ptv3_ops.new_amax)
        oi = point.order_type[self.attn.order_index]
        if h is not None:
            qkv, q_amax = ops.linear(h, self.attn.qkv.weight, self.attn.qkv.bias, y_amax=True)
        if self.attn.enable_flash:
            K, win3, nw = point_windows_flash(point, self.attn.patch_size_max)
            a = ops.window_attention_varlen(qkv, point.order_phys[oi], win3, nw, K, self.attn.num_heads, C,
                                            qkv_amax=q_amax)
        else:
            K, win, nw = point_windows(point, self.attn.patch_size_max)
            if ops.window_attention_proj_ok(C, self.attn.num_heads):
                # attention + proj + residual in one launch: the attention output never reaches HBM (attn_proj.hip)
                x2 = ops.window_attention_proj(qkv, point.order_phys[oi], win, nw, K, self.attn.num_heads, C,
                                               self.attn.proj, x1, q_amax)
                return self._mlp_tail(point, x2, out, rowexp=fused)
            a = ops.window_attention(qkv, point.order_phys[oi], win, nw, K, self.attn.num_heads, C, qkv_amax=q_amax)
        x2 = ops.linear(a, self.attn.proj.weight, self.attn.proj.bias, residual=x1)
        return self._mlp_tail(point, x2, out, rowexp=fused)

    def _mlp_tail(self, point: Point, x2: Tensor, out: Optional[Tensor], rowexp: bool = False) -> Point:
        """x += MLP(LN2 x) (calflops.py:72-82).  rowexp: also emit the output rows' fused-conv exponents (this map
        runs the fused SubM conv, so the next Block on it reads them instead of re-reading its input)."""
        ln2 = self.norm2[0]
        mlp = self.mlp[0]
        point.pop("feat_rowexp", None)
        if ops.block_mlp_ok(x2, self.channels):  # norm2 -> fc1 -> GELU -> fc2 -> + shortcut in one launch (mlp.hip)
            e = torch.empty(x2.shape[0], device=x2.device, dtype=torch.int32) if rowexp else None
            point.feat = ops.block_mlp(x2, ln2, mlp.fc1, mlp.fc2, out=out, rowexp=e)
            if e is not None:
                point.feat_rowexp = (point.feat, e)
            return point
        h2 = ops.layernorm(x2, ln2.weight, ln2.bias, ln2.eps)
        m = ops.linear(h2, mlp.fc1.weight, mlp.fc1.bias, act=ops.ACT_GELU)
        point.feat = ops.linear(m, mlp.fc2.weight, mlp.fc2.bias, residual=x2, out=out)
        return point


def bn_affine(bn: nn.BatchNorm1d):
    """Eval BatchNorm1d as per-channel (scale, shift): y = x*scale + shift (cached until a tensor changes)."""
    ts = (bn.weight, bn.bias, bn.running_mean, bn.running_var)
    key = tuple((t.data_ptr(), t._version) for t in ts) + (bn.eps,)
    cache = getattr(bn, "_sfx_affine", None)
    if cache is not None and cache[0] == key:
        return cache[1]
    with torch.no_grad():
        scale = bn.weight / torch.sqrt(bn.running_var + bn.eps)
        shift = bn.bias - bn.running_mean * scale
    val = (scale.detach().contiguous(), shift.detach().contiguous())
    object.__setattr__(bn, "_sfx_affine", (key, val))
    return val


class SerializedPooling(nn.Module):
    def __init__(self, in_channels, out_channels, stride=2, norm_layer=None, act_layer=None):
        super().__init__()
        assert stride == 2 ** (math.ceil(stride) - 1).bit_length()
        self.stride = stride
        self.proj = nn.Linear(in_channels, out_channels)
        self.norm = PointSequential(norm_layer(out_channels))
        self.act = PointSequential(act_layer())

    def pooling_depth(self, depth: int) -> int:
        """Pointcept's pooling_depth (ceil(stride) - 1).bit_length(), 0 when it exceeds the serialized depth."""
        pd = (math.ceil(self.stride) - 1).bit_length()
        return 0 if pd > depth else pd

    def _pd(self, point: Point) -> int:
        return self.pooling_depth(point.serialized_depth)

    def geometry_begin(self, point: Point):
        return ops.pool_geometry_begin(point.codes_phys, point.order_phys, self._pd(point))

    def geometry_end(self, point: Point, perm: Sequence[int], state, m: Optional[int] = None,
                     deferred: Optional[list] = None, pairs: bool = True, centre: bool = False):
        """The integer half of SerializedPooling.forward: clusters (code >> 3*pd, unique), their members
        (sidx / idx_ptr CSR), the pooled coords, codes, orders and neighbour map.  -> (new Point, sidx, idx_ptr, m)
        m: the cluster count when already known (PointTransformerV3.forward's pool_counts_begin)."""
        pd = self._pd(point)
        depth = point.serialized_depth - pd
        code_bits = point.code_bits - 3 * pd
        sidx, cluster, idx_ptr, m, codes, order, inverse, grid, batch = ops.pool_geometry_end(
            state, point.codes_phys, point.order_phys, point.order_type[0], pd, point.grid_coord, point.get("batch"),
            point.code_bits, m=m, deferred=deferred)
        coord = ops.segment_mean(point.coord, idx_ptr, sidx, m)
        new = Point(coord=coord, grid_coord=grid, codes_phys=codes, order_phys=order,
                    inverse_phys=inverse, order_type=[point.order_type[p] for p in perm],
                    serialized_depth=depth, code_bits=code_bits, pooling_inverse=cluster, pooling_parent=point)
        if batch is not None:
            new.batch = batch
            new.offset = torch.cumsum(torch.bincount(batch.long().cpu(), minlength=len(point.offset)), 0).tolist()
        else:
            new.offset = [m]
        new.nbr = ops.subm_neighbors(grid, new.get("batch"), with_pairs=pairs, centre=centre)
        return new, sidx, idx_ptr, m

    def geometry(self, point: Point, perm: Sequence[int]):
        return self.geometry_end(point, perm, self.geometry_begin(point))

    def run(self, point: Point, perm: Sequence[int], m: Optional[int] = None, deferred: Optional[list] = None,
            pairs: bool = True, centre: bool = False) -> Point:
        st = self.geometry_begin(point)
        # the projection does not depend on the clusters: enqueued while the host waits for the pooled count
        pf = ops.linear(point.feat, self.proj.weight, self.proj.bias)
        new, sidx, idx_ptr, m = self.geometry_end(point, perm, st, m, deferred, pairs=pairs, centre=centre)
        sc, sh = bn_affine(self.norm[0])
        new.feat = ops.segment_max_affine_act(pf, idx_ptr, sidx, m, sc, sh, ops.ACT_GELU)
        return new


class SerializedUnpooling(nn.Module):
    def __init__(self, in_channels, skip_channels, out_channels, norm_layer=None, act_layer=None):
        super().__init__()
        self.proj = PointSequential(nn.Linear(in_channels, out_channels), norm_layer(out_channels), act_layer())
        self.proj_skip = PointSequential(nn.Linear(skip_channels, out_channels), norm_layer(out_channels),
                                         act_layer())

    def run(self, point: Point) -> Point:
        parent = point.pop("pooling_parent")
        inverse = point.pop("pooling_inverse")
        sc, sh = bn_affine(self.proj[1])
        coarse = ops.linear(point.feat, self.proj[0].weight, self.proj[0].bias, scale=sc, shift=sh, act=ops.ACT_GELU)
        sc2, sh2 = bn_affine(self.proj_skip[1])
        skip = torch.empty(parent.feat.shape[0], coarse.shape[1], device=coarse.device)
        parent.feat = ops.linear(
            parent.feat, self.proj_skip[0].weight, self.proj_skip[0].bias, scale=sc2, shift=sh2, act=ops.ACT_GELU,
            residual=coarse, residual_idx=inverse, pre_out=skip)
        # Pointcept quirk: SerializedUnpooling does not refresh sparse_conv_feat, so the next Block's
        # SubMConv3d sees proj_skip(parent) only (PointSequential semantics, pointtransformer_v3.py:52-79)
        parent.stale_conv_feat = skip
        return parent


def point_windows(point: Point, patch_size_max: int):
    """K = min(min bincount, patch_size_max) and the device window table (cached per Point)."""
    counts = [b - a for a, b in zip([0] + list(point.offset[:-1]), point.offset)]
    K = min(min(counts), patch_size_max)
    key = ("win", K)
    if key not in point:
        t = torch.from_numpy(ops.window_table_np(point.offset, K)).pin_memory()
        point[key] = (t.to(point.feat.device, non_blocking=True), t.shape[0])  # no queue drain
    win, nw = point[key]
    return K, win, nw


def point_windows_flash(point: Point, patch_size_max: int):
    """Flash mode: K = patch_size_max and the (key_start, query_start, key_count) device table (cached per Point)."""
    K = patch_size_max
    key = ("winv", K)
    if key not in point:
        t = torch.from_numpy(ops.window_table_varlen_np(point.offset, K)).pin_memory()
        point[key] = (t.to(point.feat.device, non_blocking=True), t.shape[0])
    win3, nw = point[key]
    return K, win3, nw


class _Container(nn.Module):
    def add(self, module, name):
        self.add_module(name, module)


class PointTransformerV3(nn.Module):
    def __init__(self, in_channels=6, order=ORDERS, stride=(2, 2, 2, 2), enc_depths=(2, 2, 2, 6, 2),
                 enc_channels=(32, 64, 128, 256, 512), enc_num_head=(2, 4, 8, 16, 32),
                 enc_patch_size=(48, 48, 48, 48, 48), dec_depths=(2, 2, 2, 2), dec_channels=(64, 64, 128, 256),
                 dec_num_head=(4, 4, 8, 16), dec_patch_size=(48, 48, 48, 48), mlp_ratio=4, turn_off_bn=False,
                 shuffle_orders=True, embedding_type="MLP", drop_path=0.3, enable_flash=False):
        super().__init__()
        if turn_off_bn:
            raise NotImplementedError("turn_off_bn=True is not on the SplatFormer path (ptv3_base.gin:30)")
        if embedding_type != "MLP":
            raise NotImplementedError("only embedding_type='MLP' (ptv3_base.gin:32) is on the path")
        self.num_stages = len(enc_depths)
        self.order = [order] if isinstance(order, str) else list(order)
        self.shuffle_orders = shuffle_orders
        self.enc_channels, self.dec_channels = list(enc_channels), list(dec_channels)
        assert self.num_stages == len(stride) + 1 == len(enc_channels) == len(enc_num_head)
        bn_layer = lambda c: nn.BatchNorm1d(c, eps=1e-3, momentum=0.01)
        self.embedding = PointSequential(nn.Linear(in_channels, enc_channels[0]), bn_layer(enc_channels[0]),
                                         nn.GELU())
        self.enc = _Container()
        for s in range(self.num_stages):
            enc = _Container()
            if s > 0:
                enc.add(SerializedPooling(enc_channels[s - 1], enc_channels[s], stride[s - 1], bn_layer, nn.GELU),
                        "down")
            for i in range(enc_depths[s]):
                enc.add(Block(enc_channels[s], enc_num_head[s], enc_patch_size[s], mlp_ratio, i % len(self.order),
                              f"stage{s}", enable_flash), f"block{i}")
            self.enc.add(enc, f"enc{s}")
        # DropPath schedule (reference pointtransformer_v3.py:280-287, :330-339): linspace(0, p) over the
        # encoder blocks in order, and over the decoder blocks with each stage's slice reversed
        enc_dp = torch.linspace(0, drop_path, sum(enc_depths)).tolist()
        for s in range(self.num_stages):
            stage = getattr(self.enc, f"enc{s}")
            for i in range(enc_depths[s]):
                getattr(stage, f"block{i}").drop_prob = enc_dp[sum(enc_depths[:s]) + i]
        self.dec = _Container()
        dch = list(dec_channels) + [enc_channels[-1]]
        for s in reversed(range(self.num_stages - 1)):
            dec = _Container()
            dec.add(SerializedUnpooling(dch[s + 1], enc_channels[s], dch[s], bn_layer, nn.GELU), "up")
            for i in range(dec_depths[s]):
                dec.add(Block(dch[s], dec_num_head[s], dec_patch_size[s], mlp_ratio, i % len(self.order),
                              f"stage{s}", enable_flash), f"block{i}")
            self.dec.add(dec, f"dec{s}")
        dec_dp = torch.linspace(0, drop_path, sum(dec_depths)).tolist()
        for s in range(self.num_stages - 1):
            sl = dec_dp[sum(dec_depths[:s]):sum(dec_depths[:s + 1])][::-1]
            stage = getattr(self.dec, f"dec{s}")
            for i in range(dec_depths[s]):
                getattr(stage, f"block{i}").drop_prob = sl[i]
        self.last_perms: List[List[int]] = []

    def _draw_perm(self, perms_override, k):
        if perms_override is not None:
            p = list(perms_override[k])
        elif self.shuffle_orders:
            p = torch.randperm(len(self.order)).tolist()  # same RNG draw as Point.serialization / pooling
        else:
            p = list(range(len(self.order)))
        self.last_perms.append(p)
        return p

    def stage_needs_pairs(self, s: int, n: Optional[int] = None) -> bool:
        """Whether an eval forward reads stage s's SubM pair lists (n points): not when every Block on that map
        (encoder stage s, decoder stage s) runs the fused conv, which reads the neighbour table only."""
        chans = [self.enc_channels[s]] + ([self.dec_channels[s]] if s < len(self.dec_channels) else [])
        return not all(ops.subm_fused_ok(c, n) for c in chans)

    def prepare(self, data_dict, perms: Optional[List[Sequence[int]]] = None, pairs: bool = True,
                reorder: bool = False, centre_pairs: bool = False) -> Point:
        """Point + serialization (randperm draw 0) + stage-0 neighbour map; `feat` is not embedded yet.

        reorder: renumber the points by their first serialized order (sfx_serialize_permute; `point.perm[i]` is the
        input row of point i) so every stage-0 gather -- SubM neighbours, attention windows, pooling clusters --
        reads neighbouring rows; the caller permutes `feat` the same way and scatters the output back.  The
        results are those of the input numbering: serialization ties (points of one voxel) keep their input
        order, so the lowest-index voxel representative and every stable sort are unchanged."""
        feat = data_dict["feat"]
        _lib.require_gpu(feat)
        dev = feat.device
        offset = data_dict["offset"]
        offset = offset.tolist() if isinstance(offset, Tensor) else list(offset)
        grid = data_dict["grid_coord"]
        grid = grid if grid.dtype == torch.int32 else grid.int()
        grid = grid.contiguous()
        n = feat.shape[0]
        B = len(offset)
        batch = None
        if B > 1:
            batch = torch.empty(n, device=dev, dtype=torch.int32)
            offs = torch.tensor(offset, dtype=torch.int64, device=dev)
            _lib.call("sfx_offsets_to_batch", n, B, offs.data_ptr(), batch.data_ptr(), _lib.stream())
        # the stage-0 neighbour map needs no serialization: enqueued before the depth read, it keeps the GPU busy
        # while the host enqueues the serialization (the read drains the queue up to the grid max's copy)
        nbr = None if (reorder or not NBR_EARLY) else ops.subm_neighbors(grid, batch, with_pairs=pairs,
                                                                          centre=centre_pairs)
        d = data_dict.get("serialized_depth")
        if isinstance(d, _lib.HostRead):  # the grid max, read back while the embedding runs
            depth = int(d.get()[0]).bit_length()
        else:
            depth = int(d) if d is not None else int(grid.max().item()).bit_length()
        assert depth * 3 + len(offset).bit_length() <= 63 and depth <= 16
        code_bits = 3 * depth + max(0, (B - 1).bit_length())
        self.last_perms = []
        codes, order, inverse = ops.serialize(grid, batch, depth, code_bits, self.order)
        p0 = self._draw_perm(perms, 0)
        coord = data_dict["coord"].float().contiguous()
        perm = None
        if reorder and batch is None:
            perm = order[0]
            codes, order, inverse, grid, coord = ops.serialize_permute(codes, order, inverse, grid, coord)
        point = Point(coord=coord, grid_coord=grid, offset=offset, codes_phys=codes,
                      order_phys=order, inverse_phys=inverse, order_type=p0, serialized_depth=depth,
                      code_bits=code_bits)
        if perm is not None:
            point.perm = perm
        if batch is not None:
            point.batch = batch
        point.nbr = nbr if nbr is not None else ops.subm_neighbors(grid, batch, with_pairs=pairs, centre=centre_pairs)
        return point

    @torch.no_grad()
    def forward(self, data_dict, perms: Optional[List[Sequence[int]]] = None, out: Optional[Tensor] = None,
                reorder: bool = False) -> Point:
        """reorder (prepare): the backbone runs on the points renumbered by serialized order; the returned Point's
        `perm` maps its rows to the input rows, and `out` (if given) receives the features in INPUT order."""
        feat = data_dict["feat"]
        _lib.require_gpu(feat)
        emb, bnm = self.embedding[0], self.embedding[1]
        sc, sh = bn_affine(bnm)
        # the embedding needs no geometry: enqueued first, it runs while prepare() waits for the grid depth
        if ops.point_embed_ok(feat, emb.weight):
            emb_feat = ops.point_embed(feat, emb.weight, emb.bias, sc, sh)
        else:
            emb_feat = ops.linear(feat, emb.weight, emb.bias, scale=sc, shift=sh, act=ops.ACT_GELU)
        # eval maps list the centre offset with the pairs: one pair launch per SubM conv (ops.SUBM_CENTRE_PAIRS)
        cp = ops.SUBM_CENTRE_PAIRS
        point = self.prepare(data_dict, perms, pairs=self.stage_needs_pairs(0, feat.shape[0]), reorder=reorder,
                             centre_pairs=cp)
        perm = point.get("perm")
        point.feat = emb_feat if perm is None else ops.move_rows(emb_feat, perm)
        final_out = out
        if perm is not None:
            out = None  # the last Block writes the renumbered rows; scattered into final_out below
        # every pooling's cluster count from the stage-0 codes, read back while stage 0 runs: no pooling waits
        pools = [getattr(self.enc, f"enc{s}").down for s in range(1, self.num_stages)]
        shifts, depth, cum = [], point.serialized_depth, 0
        for mod in pools:  # the same pooling depths the poolings themselves will use (SerializedPooling._pd)
            pd = mod.pooling_depth(depth)
            depth, cum = depth - pd, cum + pd
            shifts.append(3 * cum)
        counts_rd = ops.pool_counts_begin(point.codes_phys, point.order_phys, shifts) if POOL_COUNTS_UPFRONT else None
        self.check_deferred(wait=True)  # the previous forward's pooling checks (long complete by now)
        self._forward_id = self.__dict__.get("_forward_id", 0) + 1
        deferred: list = []
        k = 1
        for s in range(self.num_stages):
            stage = getattr(self.enc, f"enc{s}")
            for name, mod in stage.named_children():
                if name == "down":
                    m = counts_rd.get()[k - 1] if counts_rd is not None else None
                    point = mod.run(point, self._draw_perm(perms, k), m=m, deferred=deferred,
                                    pairs=self.stage_needs_pairs(s, m), centre=cp)
                    k += 1
                else:
                    point = mod.run(point)
        dec_names = [f"dec{s}" for s in reversed(range(self.num_stages - 1))]
        for di, dn in enumerate(dec_names):
            stage = getattr(self.dec, dn)
            children = list(stage.named_children())
            for ci, (name, mod) in enumerate(children):
                if name == "up":
                    point = mod.run(point)
                else:
                    conv_in = point.pop("stale_conv_feat", None)
                    last = di == len(dec_names) - 1 and ci == len(children) - 1
                    point = mod.run(point, conv_in=conv_in, out=out if last else None)
        # the pooling run-count checks whose reads have landed run now; the rest when the caller consumes the
        # result (FeaturePredictor.check_refine, evaluate_scenes) or at the next forward: waiting here would hold
        # back the launches the caller enqueues after the backbone (the heads, the render) until the whole
        # backbone has run -- a drained queue at every refine
        fid = self._forward_id
        self._deferred = self.__dict__.get("_deferred", []) + [(rd, m, fid, i + 1) for i, (rd, m) in
                                                                enumerate(deferred)]
        self.check_deferred(wait=False)
        if perm is not None and final_out is not None:
            ops.move_rows(point.feat, perm, dst=final_out, scatter=True)
        return point

    def check_deferred(self, wait: bool = True) -> None:
        """Validate the pooled run counts read back asynchronously by forward (pool_geometry_end's `deferred`).

        Every entry is taken off the pending list before it is validated, so a failing forward raises exactly
        once (naming its forward id and pooling) and later forwards are checked on their own.  An entry whose
        read has not landed stays pending unless `wait`."""
        pending, errors = [], []
        for rd, m, fid, k in self.__dict__.get("_deferred", []):
            if not (wait or rd.ready()):
                pending.append((rd, m, fid, k))
                continue
            try:
                ops.check_pool_runs(rd.get(), m)
            except RuntimeError as e:
                errors.append(f"forward {fid}, pooling {k}: {e}")
        self._deferred = pending
        if errors:
            raise RuntimeError("; ".join(errors))


class PointTransformerV3Model(nn.Module):
    """reference models/pointtransformer_v3.py:81-182 (gin-configurable assembly), ptv3_base.gin defaults."""

    def __init__(self, in_channels, enable_flash=False, enc_dim=64, output_dim=96, turn_off_bn=False,
                 stride=(1, 2, 2, 2), embedding_type="MLP", enc_depths=(2, 2, 2, 6, 2), enc_num_head=(2, 4, 8, 16, 32),
                 dec_depths=(2, 2, 2, 2), dec_num_head=(4, 4, 8, 16), dec_channels=None, enc_channels=None,
                 pdnorm_bn=False, pdnorm_ln=False, pretrained_ckpt=None, additional_info=None):
        super().__init__()
        if pdnorm_bn or pdnorm_ln:
            raise NotImplementedError("PDNorm is not on the SplatFormer path")
        if additional_info and additional_info.get("tome") not in (None, "base") or \
                (additional_info and float(additional_info.get("r", 0.0)) != 0.0):
            raise NotImplementedError("token merging variants are out of scope (SURVEY.md §2); base r=0 only")
        if dec_channels is None:
            dec_channels = {64: (64, 64, 128, 256), 128: (128, 128, 256, 256), 96: (96, 96, 128, 256)}.get(output_dim)
            if dec_channels is None:
                raise ValueError("Unsupported output_dim")
        if enc_channels is None:
            enc_channels = {32: (32, 64, 128, 256, 512), 64: (64, 96, 128, 256, 512)}.get(enc_dim)
            if enc_channels is None:
                raise ValueError("Unsupported enc_dim")
        self.dec_channels = tuple(dec_channels)
        # enable_flash: K = 1024 windows cut at cu_seqlens (sfx_window_attention_varlen), fp32 arithmetic where
        # Pointcept's flash-attn call runs fp16 (>= the reference's precision)
        patch = 1024 if enable_flash else 128
        self.backbone = PointTransformerV3(
            in_channels=in_channels, order=ORDERS, stride=stride, enc_depths=enc_depths, enc_channels=enc_channels,
            enc_num_head=enc_num_head, enc_patch_size=(patch,) * len(enc_channels), dec_depths=dec_depths,
            dec_channels=dec_channels, dec_num_head=dec_num_head, dec_patch_size=(patch,) * len(dec_channels),
            mlp_ratio=4, turn_off_bn=turn_off_bn, shuffle_orders=True, embedding_type=embedding_type,
            enable_flash=enable_flash)
        self.enable_flash = enable_flash
        self.output_dim = self.dec_channels[0]
        if pretrained_ckpt is not None:
            sd = torch.load(pretrained_ckpt, map_location="cpu", weights_only=True)["state_dict"]
            sd = {k.replace("module.backbone.", ""): v for k, v in sd.items() if "backbone." in k}
            own = self.backbone.state_dict()
            load = {k: v for k, v in sd.items() if k in own and own[k].shape == v.shape}
            self.backbone.load_state_dict(load, strict=False)

    def forward(self, x, perms=None, out=None, reorder=False):
        return self.backbone(x, perms=perms, out=out, reorder=reorder)
