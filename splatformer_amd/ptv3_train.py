"""Training forward + hand-written backward of the refiner (configs C/D) on libsfx HIP kernels.

Reference: train.py:236-303 trains FeaturePredictor with `model.train()` semantics --
- DropPath (timm, per point) on the attention and MLP branches with the schedule of
  pointtransformer_v3.py:280-339 (drop_path=0.3, :145);
- BatchNorm1d with batch statistics (SyncBatchNorm under DDP, train.py:404) in the embedding, the pooling
  and the unpooling projections, running statistics updated;
- the same randperm(4) order shuffles as evaluation;
and only the parameters whose name contains 'attn.qkv' require grad (utils/optimizers.py:48-52
`finetune_list=['attn.qkv']; filter_grads(...)`).  The backward therefore propagates the input gradient
through every layer from the loss down to the first encoder block, and accumulates weight/bias gradients
for the qkv projections only.

The forward keeps per-layer state on a tape (saved activations, not an autograd graph); `backward`
replays it in reverse.  Every op is a libsfx kernel (train_ops / ptv3_ops); torch only allocates.
"""
from __future__ import annotations

import os
from typing import Callable, Dict, List, Optional, Sequence

import torch
from torch import Tensor

from . import ptv3_ops as ops
from . import train_ops as tops
from .ptv3 import (Block, Point, PointTransformerV3, SerializedPooling, SerializedUnpooling, point_windows,
                   point_windows_flash)

MaskFn = Callable[[str, int, float], Optional[Tensor]]


def wt(w: Tensor) -> Tensor:
    """W^T of a [N, K...] weight (flattened to [N, K]), cached on the tensor that owns the storage until the
    weight changes (the cache lives and dies with that tensor, so a reused allocation never hits it)."""
    holder = w._base if w._base is not None else w
    w2 = w.detach().reshape(w.shape[0], -1)
    key = (w2.storage_offset(), tuple(w2.shape), w2.stride(0), w._version)
    cache = holder.__dict__.setdefault("_sfx_wt", {})
    t = cache.get(key)
    if t is None:
        if len(cache) > 64:
            cache.clear()
        t = tops.transpose(w2)
        cache[key] = t
    return t


_MASK_STREAMS = [0]  # DropMasks objects created in this process (each gets its own seed stream)


class DropMasks:
    """timm DropPath per point: keep ~ Bernoulli(1-p), scaled by 1/(1-p); None when p == 0 (Identity).  One
    sfx_drop_mask launch per mask, hash-seeded from (base seed, rank, stream id, draw counter): reproducible for a
    seeded generator with no device read, different on every DDP rank (timm draws each rank's masks from its own
    device RNG state), and different for every DropMasks of the process (a second Trainer, or one re-created in
    the same process, does not replay the first one's masks).  state_dict / load_state_dict carry the counter
    across a checkpoint resume (Trainer.state_dict)."""

    def __init__(self, generator: Optional[torch.Generator] = None, rank: Optional[int] = None):
        self.base = int(generator.initial_seed()) if generator is not None else int(torch.initial_seed())
        if rank is None:
            dist = torch.distributed
            rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        self.rank = int(rank)
        self.stream_id = _MASK_STREAMS[0]
        _MASK_STREAMS[0] += 1
        self.k = 0

    def seed(self) -> int:
        m = 0xFFFFFFFFFFFFFFFF
        s = (self.base * 0x9E3779B97F4A7C15) & m
        s = (s ^ ((self.rank + 1) * 0xBF58476D1CE4E5B9)) & m
        s = (s ^ (self.stream_id * 0x94D049BB133111EB)) & m
        return (s + self.k * 0xD1B54A32D192ED03) & m

    def __call__(self, name: str, n: int, p: float, device=None) -> Optional[Tensor]:
        if p <= 0.0:
            return None
        self.k += 1
        return tops.drop_mask(n, 1.0 - p, self.seed(), device)

    def state_dict(self) -> dict:
        return {"base": self.base, "rank": self.rank, "stream_id": self.stream_id, "k": self.k}

    def load_state_dict(self, sd: dict) -> None:
        self.base, self.rank, self.stream_id, self.k = (int(sd[k]) for k in ("base", "rank", "stream_id", "k"))


def device_drop_masks(generator: Optional[torch.Generator] = None, rank: Optional[int] = None) -> MaskFn:
    """The default DropPath mask source of the training step (DropMasks)."""
    return DropMasks(generator, rank)


def _grad_buffers(lin: torch.nn.Linear):
    for p in (lin.weight, lin.bias):
        if p is not None and p.requires_grad and p.grad is None:
            p.grad = torch.zeros_like(p)
    return (lin.weight.grad if lin.weight.requires_grad else None,
            lin.bias.grad if lin.bias is not None and lin.bias.requires_grad else None)


# ---- Block ------------------------------------------------------------------------------------------------
# SFX_MLP_TRAIN_FUSED=0: the training MLP tail as LayerNorm + two GEMMs forward and two GEMMs backward (the [n, 4C]
# GELU output and hidden gradient through HBM) instead of sfx_block_mlp_train / sfx_block_mlp_bwd
MLP_TRAIN_FUSED = os.environ.get("SFX_MLP_TRAIN_FUSED", "1") != "0"


def mlp_train_fused_ok(x2: Tensor, C: int) -> bool:
    return MLP_TRAIN_FUSED and C in ops.MLP_CHANNELS and x2.is_contiguous() and x2.data_ptr() % 16 == 0
def block_forward(blk: Block, name: str, point: Point, masks: MaskFn, conv_in: Optional[Tensor] = None,
                  out: Optional[Tensor] = None) -> dict:
    x = point.feat
    n, C = x.shape
    ln_c = blk.cpe[2]
    ln1, ln2, mlp = blk.norm1[0], blk.norm2[0], blk.mlp[0]
    wf, bf = blk.cpe_fused()  # Linear folded into the conv (frozen in training: filter_grads(['attn.qkv']))
    u = ops.subm_conv(x if conv_in is None else conv_in, point.nbr, wf, bf)
    x1, h = ops.cpe_residual_ln(u, x, ln_c.weight, ln_c.bias, ln1.weight, ln1.bias, ln1.eps)
    qkv = ops.linear(h, blk.attn.qkv.weight, blk.attn.qkv.bias)
    order = point.order_phys[point.order_type[blk.attn.order_index]]
    if blk.attn.enable_flash:  # K = 1024 windows cut at cu_seqlens
        K, win, nw = point_windows_flash(point, blk.attn.patch_size_max)
        a = ops.window_attention_varlen(qkv, order, win, nw, K, blk.attn.num_heads, C)
    else:
        K, win, nw = point_windows(point, blk.attn.patch_size_max)
        a = ops.window_attention(qkv, order, win, nw, K, blk.attn.num_heads, C)
    ma = masks(name + ".attn", n, blk.drop_prob, x.device)
    x2 = ops.linear(a, blk.attn.proj.weight, blk.attn.proj.bias, residual=x1, rowscale=ma)
    z = torch.empty(n, mlp.fc1.weight.shape[0], device=x.device, dtype=torch.float32)
    mm = masks(name + ".mlp", n, blk.drop_prob, x.device)
    fused = mlp_train_fused_ok(x2, C)
    if fused:  # LN2 + fc1 (z stored) + GELU + fc2 + mask + residual in one launch (csrc/mlp.hip MLP_TRAIN)
        point.feat = ops.block_mlp_train(x2, ln2, mlp.fc1, mlp.fc2, z, rowscale=mm, out=out)
    else:
        h2 = ops.layernorm(x2, ln2.weight, ln2.bias, ln2.eps)
        m = ops.linear(h2, mlp.fc1.weight, mlp.fc1.bias, act=ops.ACT_GELU, pre_out=z, pre_before_act=True)
        del h2
        point.feat = ops.linear(m, mlp.fc2.weight, mlp.fc2.bias, residual=x2, rowscale=mm, out=out)
    return dict(kind="block", blk=blk, name=name, u=u, x1=x1, h=h, qkv=qkv, a=a, x2=x2, z=z, ma=ma, mm=mm,
                order=order, win=win, nw=nw, K=K, smap=point.nbr, sep_conv_in=conv_in is not None, mlp_fused=fused)


_TRACE: Optional[list] = None  # debugging: set to a list to record (tag, tensor) of the backward


def _trace(tag: str, t: Optional[Tensor]) -> None:
    if _TRACE is not None and t is not None:
        _TRACE.append((tag, t.detach().clone()))


def block_backward(rec: dict, dy: Tensor, need_input: bool):
    """-> (d block input, d separate conv input or None); qkv weight/bias grads accumulated."""
    blk: Block = rec["blk"]
    nm = rec["name"]
    for k in ("u", "x1", "h", "qkv", "x2", "z"):
        _trace(f"{nm}.fwd.{k}", rec[k])
    _trace(f"{nm}.dy", dy)
    C = blk.channels
    ln_c = blk.cpe[2]
    ln1, ln2, mlp = blk.norm1[0], blk.norm2[0], blk.mlp[0]
    if rec.get("mlp_fused"):  # fc2^T, GELU', fc1^T in one launch: the [n, 4C] hidden gradient stays on chip
        dh2 = ops.block_mlp_bwd(dy, ln2, mlp.fc1, mlp.fc2, rec["z"], rowscale=rec["mm"])
    else:
        dm = tops.linear_bwd_data(dy, wt(mlp.fc2.weight), rowscale=rec["mm"], dact=tops.DACT_GELU, dact_pre=rec["z"])
        dh2 = tops.linear_bwd_data(dm, wt(mlp.fc1.weight))
        _trace(f"{nm}.dm", dm)
        del dm
    dx2 = tops.layernorm_bwd(rec["x2"], ln2.weight, dh2, ln2.eps, dres=dy)
    _trace(f"{nm}.dh2", dh2)
    _trace(f"{nm}.dx2", dx2)
    del dh2
    da = tops.linear_bwd_data(dx2, wt(blk.attn.proj.weight), rowscale=rec["ma"])
    if blk.attn.enable_flash:
        dqkv = tops.window_attention_varlen_bwd(rec["qkv"], rec["order"], rec["win"], rec["nw"], rec["K"],
                                                blk.attn.num_heads, C, da)
    else:
        dqkv = tops.window_attention_bwd(rec["qkv"], rec["order"], rec["win"], rec["nw"], rec["K"],
                                         blk.attn.num_heads, C, da, attn_out=rec["a"])
    _trace(f"{nm}.da", da)
    _trace(f"{nm}.dqkv", dqkv)
    del da
    gw, gb = _grad_buffers(blk.attn.qkv)
    if gw is not None:
        tops.linear_wgrad(dqkv, rec["h"], gw, gb)
    elif gb is not None:
        raise NotImplementedError("qkv bias trainable without its weight")
    if not need_input:
        return None, None
    dh = tops.linear_bwd_data(dqkv, wt(blk.attn.qkv.weight))
    del dqkv
    dx1, du = tops.cpe_ln_bwd(rec["u"], rec["x1"], ln_c.weight, ln1.weight, dx2, dh, ln1.eps)
    del dh, dx2
    dt = du
    wct = wt(blk.cpe_fused()[0])  # fused [Cout, 27*Cin] -> [27*Cin, Cout]
    if rec["sep_conv_in"]:
        dci = torch.zeros_like(dx1)
        tops.subm_conv_bwd_data(dt, rec["smap"], wct, dci)
        return dx1, dci
    tops.subm_conv_bwd_data(dt, rec["smap"], wct, dx1)  # residual gradient + conv gradient
    return dx1, None


# ---- pooling / unpooling -----------------------------------------------------------------------------------
def pool_forward(pool: SerializedPooling, point: Point, perm: Sequence[int], group=None):
    new, sidx, idx_ptr, m = pool.geometry(point, perm)
    pf = ops.linear(point.feat, pool.proj.weight, pool.proj.bias)
    s, arg = tops.segment_max_arg(pf, idx_ptr, sidx, m)
    del pf
    new.feat, st = tops.bn_train_forward(s, pool.norm[0], ops.ACT_GELU, group=group)
    new.pool_sidx, new.pool_idx_ptr = sidx, idx_ptr
    return new, dict(kind="pool", mod=pool, arg=arg, st=st, n_parent=point.feat.shape[0], group=group)


def pool_backward(rec: dict, dfeat: Tensor) -> Tensor:
    pool: SerializedPooling = rec["mod"]
    ds = tops.bn_act_bwd(rec["st"], pool.norm[0], ops.ACT_GELU, dfeat, group=rec["group"])
    dpf = tops.segment_max_bwd(ds, rec["arg"], rec["n_parent"])
    return tops.linear_bwd_data(dpf, wt(pool.proj.weight))


def unpool_forward(up: SerializedUnpooling, point: Point, group=None):
    parent = point.pop("pooling_parent")
    inverse = point.pop("pooling_inverse")
    zc = ops.linear(point.feat, up.proj[0].weight, up.proj[0].bias)
    coarse, stc = tops.bn_train_forward(zc, up.proj[1], ops.ACT_GELU, group=group)
    zs = ops.linear(parent.feat, up.proj_skip[0].weight, up.proj_skip[0].bias)
    skip, sts = tops.bn_train_forward(zs, up.proj_skip[1], ops.ACT_GELU, group=group)
    parent.feat = tops.bn_apply(sts, ops.ACT_GELU, residual=coarse, residual_idx=inverse)
    parent.stale_conv_feat = skip  # Pointcept quirk (see SerializedUnpooling.run)
    rec = dict(kind="unpool", mod=up, stc=stc, sts=sts, sidx=point.pool_sidx, idx_ptr=point.pool_idx_ptr,
               m=point.feat.shape[0], group=group)
    return parent, rec


def unpool_backward(rec: dict, dfeat: Tensor, dstale: Optional[Tensor]):
    """-> (d coarse input feature, d encoder skip feature)"""
    up: SerializedUnpooling = rec["mod"]
    dskip = dfeat if dstale is None else dfeat + dstale
    dcoarse = tops.segment_sum(dfeat, rec["idx_ptr"], rec["sidx"], rec["m"])
    dzs = tops.bn_act_bwd(rec["sts"], up.proj_skip[1], ops.ACT_GELU, dskip, group=rec["group"])
    d_enc = tops.linear_bwd_data(dzs, wt(up.proj_skip[0].weight))
    del dzs
    dzc = tops.bn_act_bwd(rec["stc"], up.proj[1], ops.ACT_GELU, dcoarse, group=rec["group"])
    d_coarse_in = tops.linear_bwd_data(dzc, wt(up.proj[0].weight))
    return d_coarse_in, d_enc


# ---- whole backbone ---------------------------------------------------------------------------------------
def check_trainable(bb: PointTransformerV3) -> None:
    bad = [n for n, p in bb.named_parameters() if p.requires_grad and "attn.qkv" not in n]
    if bad:
        raise NotImplementedError(
            "the training backward accumulates grads for the attn.qkv parameters only (the reference's "
            f"utils/optimizers.py:48-52 filter); these also require grad: {bad[:4]}...")


def backbone_forward(bb: PointTransformerV3, data_dict, masks: MaskFn, perms=None, out: Optional[Tensor] = None,
                     group=None):
    """PointTransformerV3.forward in train mode; -> (Point, tape)."""
    point = bb.prepare(data_dict, perms)
    emb, bnm = bb.embedding[0], bb.embedding[1]
    z = ops.linear(data_dict["feat"], emb.weight, emb.bias)
    point.feat, _ = tops.bn_train_forward(z, bnm, ops.ACT_GELU, group=group)
    del z
    enc_recs: List[List[dict]] = []
    k = 1
    for s in range(bb.num_stages):
        stage = getattr(bb.enc, f"enc{s}")
        recs = []
        for name, mod in stage.named_children():
            if name == "down":
                point, r = pool_forward(mod, point, bb._draw_perm(perms, k), group)
                k += 1
            else:
                r = block_forward(mod, f"enc.enc{s}.{name}", point, masks)
            recs.append(r)
        enc_recs.append(recs)
    dec_recs: List[List[dict]] = []
    dec_names = [f"dec{s}" for s in reversed(range(bb.num_stages - 1))]
    for di, dn in enumerate(dec_names):
        stage = getattr(bb.dec, dn)
        children = list(stage.named_children())
        recs = []
        for ci, (name, mod) in enumerate(children):
            if name == "up":
                point, r = unpool_forward(mod, point, group)
            else:
                conv_in = point.pop("stale_conv_feat", None)
                last = di == len(dec_names) - 1 and ci == len(children) - 1
                r = block_forward(mod, f"dec.{dn}.{name}", point, masks, conv_in=conv_in, out=out if last else None)
            recs.append(r)
        dec_recs.append(recs)
    return point, dict(enc=enc_recs, dec=dec_recs)


def backbone_backward(tape: dict, dout: Tensor) -> None:
    """Accumulate the qkv gradients of d(loss)/d(backbone output) = dout."""
    g = dout
    skip_grads: Dict[int, Tensor] = {}
    n_dec = len(tape["dec"])
    for di in reversed(range(n_dec)):        # dec0 (last executed) first
        recs = tape["dec"][di]
        s = n_dec - 1 - di                   # decoder stage index (dec3 executed first)
        dstale = None
        for r in reversed(recs):
            if r["kind"] == "block":
                g, dci = block_backward(r, g, need_input=True)
                if dci is not None:
                    dstale = dci
            else:
                g, skip_grads[s] = unpool_backward(r, g, dstale)
    for s in reversed(range(len(tape["enc"]))):
        if s in skip_grads:
            g = g + skip_grads.pop(s)
        recs = tape["enc"][s]
        for i, r in enumerate(reversed(recs)):
            first = i == len(recs) - 1
            if r["kind"] == "block":
                lowest = s == 0 and first
                g, _ = block_backward(r, g, need_input=not lowest)
            else:
                g = pool_backward(r, g)
