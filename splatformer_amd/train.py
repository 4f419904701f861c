"""Training step of SplatFormer on MI355X (reference train.py:236-303, configs C/D).

Per scene: FeaturePredictor forward in train mode (ptv3_train), the refined Gaussians rendered to the
training views through the gsplat-compatible autograd path (gs_render / gsplat_compat HIP kernels), the
image L1 loss `sum_v |pred_v - gt_v|.mean() / num_images / len(batch)` (train.py:272-283, image_l1 weight 1;
the LPIPS term needs VGG weights that are not available offline and is left out), backward through the
renderer to the packed refined record, then the hand-written refiner backward.  Every `accumulate_step`
micro-steps: gradient all-reduce (DDP average, one flat bucket over RCCL), clip_grad_norm_(2.0) and
Adam(lr 3e-5, eps 1e-15) on the trainable parameters (attn.qkv, utils/optimizers.py:48-52,
configs/train/default.gin).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence

import torch
from torch import Tensor

from . import _lib
from . import ptv3_ops as ops
from . import ptv3_train as pt
from . import train_ops as tops
from .dist import allreduce_mean_
from .feature_predictor import ALL_FEATURES, FeaturePredictor
from .gs_render import rasterize_gaussians_to_multiimgs


# ---- FeaturePredictor train forward / backward --------------------------------------------------------------
def refine_train(fp: FeaturePredictor, gs: Dict[str, Tensor], masks, perms=None, group=None):
    """refine_packed in train mode -> (packed [N, Cin] refined record, tape)."""
    means = gs["means"]
    dev = means.device
    n = means.shape[0]
    cin = fp.gs_features_dim
    cb = fp.backbone.output_dim
    ld = (cb + cin + 3) // 4 * 4
    h0 = torch.zeros(n, ld, device=dev, dtype=torch.float32)
    feat = h0[:, cb:cb + cin]
    grid = torch.empty(n, 3, device=dev, dtype=torch.int32)
    gmax = torch.zeros(1, device=dev, dtype=torch.int32)
    ops.gs_pack(gs, feat, float(fp.grid_resolution), grid, gmax)
    depth = int(gmax.item()).bit_length()
    data = {"coord": means, "grid_coord": grid, "offset": [n], "feat": feat, "serialized_depth": depth}
    _, bb_tape = pt.backbone_forward(fp.backbone.backbone, data, masks, perms=perms, out=h0[:, :cb], group=group)
    w1, b1, mids, wl, bl, out_dim = fp._packed_heads()
    x = h0[:, :w1.shape[1]]
    hs = [ops.linear(x, w1, b1, act=ops.ACT_RELU)]
    for wm, bm in mids:
        hs.append(ops.grouped_linear(hs[-1], wm, bm, len(fp.output_features), act=ops.ACT_RELU))
    n_tanh = fp.ch["means"] if fp.output_features[0] == "means" else 0
    o = torch.empty(n, out_dim, device=dev, dtype=torch.float32)
    packed = ops.linear(hs[-1], wl, bl, act=ops.ACT_TANH, act_ncols=n_tanh, residual=feat, pre_out=o)
    return packed, dict(bb=bb_tape, hs=hs, o=o, n_tanh=n_tanh, cb=cb)


def refine_backward(fp: FeaturePredictor, tape: dict, d_packed: Tensor) -> None:
    """d(loss)/d(packed record) -> qkv gradients (heads and the input attributes are not trained)."""
    w1, b1, mids, wl, bl, out_dim = fp._packed_heads()
    G, W = len(fp.output_features), fp.width
    hs = tape["hs"]
    dz = tops.act_bwd(d_packed.contiguous(), tape["o"], tops.DACT_TANH_OUT, ncols=tape["n_tanh"])
    dh = tops.linear_bwd_data(dz, pt.wt(wl), dact=tops.DACT_RELU, dact_pre=hs[-1])
    for li in reversed(range(len(mids))):
        wm = mids[li][0]
        prev = hs[li]
        dprev = torch.empty_like(prev)
        for g in range(G):
            sl = slice(g * W, (g + 1) * W)
            tops.linear_bwd_data(dh[:, sl], pt.wt(wm[g]), dact=tops.DACT_RELU, dact_pre=prev[:, sl], out=dprev[:, sl])
        dh = dprev
    dx = tops.linear_bwd_data(dh, pt.wt(w1))
    pt.backbone_backward(tape["bb"], dx[:, :tape["cb"]].contiguous())


def unpack_leaf(fp: FeaturePredictor, packed: Tensor, gs: Dict[str, Tensor]):
    """The refined Gaussians as views of one grad-tracking leaf (render autograd lands in leaf.grad)."""
    leaf = packed.detach().requires_grad_()
    out = fp.unpack(leaf)
    for key in ALL_FEATURES:
        if fp.sh_degree == 0 and key == "features_rest":
            continue
        if key not in out:
            out[key] = gs[key]
    return leaf, out


def image_l1(pred: Sequence[Tensor], gt: Sequence[Tensor]) -> Tensor:
    """train.py:276-283: sum over views of mean |pred - gt| (normalised by the caller)."""
    loss = None
    for p, g in zip(pred, gt):
        v = (p - g).abs().mean()
        loss = v if loss is None else loss + v
    return loss


# ---- optimiser ------------------------------------------------------------------------------------------------
class Trainer:
    """FeaturePredictor training on libsfx: filter_grads(['attn.qkv']), flat gradient bucket (one RCCL
    all-reduce per optimiser step under DDP), clip_grad_norm_ + Adam on device."""

    def __init__(self, model: FeaturePredictor, lr: float = 3e-5, eps: float = 1e-15, betas=(0.9, 0.999),
                 grad_clip_norm: float = 2.0, accumulate_step: int = 1, group=None, generator=None,
                 precision: Optional[str] = None):
        """precision: "fp32" (default; fp32-accurate refiner forward + backward) or "amp", the reference's
        `training.enable_amp` (train.py:214-299, configs/train/default.gin:11): refiner forward and backward in
        the autocast precision class (ptv3_ops.precision); the renderer, loss and optimiser stay fp32 as in the
        reference (its rasterisation runs outside the autocast region).  No loss scale: the GEMMs scale every
        operand row by its own power of two, so fp16 range limits never flush or overflow a gradient; GradScaler's
        skip of a step with non-finite gradients is kept (optimizer_step).
        Default from SFX_TRAIN_PREC."""
        self.model = model
        self.precision = precision or os.environ.get("SFX_TRAIN_PREC", "fp32")
        if self.precision not in ops.PRECISIONS:
            raise ValueError(f"precision {self.precision!r}: expected one of {sorted(ops.PRECISIONS)}")
        for name, p in model.named_parameters():       # utils/optimizers.py:4-16, :48-52
            p.requires_grad_("attn.qkv" in name)
        pt.check_trainable(model.backbone.backbone)
        self.params = [p for p in model.parameters() if p.requires_grad]
        dev = self.params[0].device
        total = sum(p.numel() for p in self.params)
        self.flat_grad = torch.zeros(total, device=dev, dtype=torch.float32)
        off = 0
        for p in self.params:
            p.grad = self.flat_grad[off:off + p.numel()].view_as(p)
            off += p.numel()
        self.exp_avg = [torch.zeros_like(p) for p in self.params]
        self.exp_avg_sq = [torch.zeros_like(p) for p in self.params]
        self.lr, self.eps, self.betas, self.clip = lr, eps, betas, grad_clip_norm
        self.accumulate_step = accumulate_step
        self.group = group
        self.world = torch.distributed.get_world_size(group) if group is not None else 1
        self.masks = pt.device_drop_masks(generator)
        self.step_count = 0
        self.skipped_steps = 0  # amp: optimiser steps skipped for non-finite gradients (GradScaler semantics)
        self.micro = 0
        self.last_norm: Optional[Tensor] = None

    def micro_step(self, scenes: List[Dict[str, Tensor]], cameras: List[dict], images: List[List[Tensor]],
                   masks=None, perms=None) -> float:
        """Forward + backward of one batch (train.py:240-289); gradients accumulate in the flat bucket."""
        self.model.train()
        masks = masks or self.masks
        total = 0.0
        num_images = sum(len(im) for im in images)  # counted over the whole batch (train.py:273-281)
        for gs, cams, imgs in zip(scenes, cameras, images):
            with ops.precision(self.precision):
                packed, tape = refine_train(self.model, gs, masks, perms=perms, group=self.group)
            leaf, out_gs = unpack_leaf(self.model, packed, gs)
            with torch.enable_grad():
                preds, _ = rasterize_gaussians_to_multiimgs(out_gs, cams)
                loss = image_l1(preds, imgs) / num_images / len(scenes) / self.accumulate_step
                loss.backward()
            with ops.precision(self.precision):
                refine_backward(self.model, tape, leaf.grad)
            total = total + loss.detach()  # summed on the device: one host read per micro-step, not per scene
            del tape, packed, leaf, out_gs, preds
        self.micro += 1
        loss = float(total)  # (drains the stream)
        _lib.check_lookback("Trainer.micro_step")  # the step's scans / radix passes (pooling, intersection sort)
        return loss

    def optimizer_step(self) -> None:
        if self.group is not None and self.world > 1:
            allreduce_mean_(self.flat_grad, self.group)  # DDP: average over ranks, one bucket
        coef = None
        if self.clip > 0:
            coef, self.last_norm = tops.grad_clip_coef([self.flat_grad], self.clip)
        if self.precision == "amp":
            # GradScaler.step (train.py:297-298) skips the optimiser step when a gradient is inf / NaN; with no loss
            # scale to halve (the per-row operand scales need none) the skip is all that remains.  One 8-byte read
            # per optimiser step: the micro-steps' loss reads have drained the stream already.
            norm = self.last_norm if self.last_norm is not None else self.flat_grad.square().sum()
            if not bool(torch.isfinite(norm).all()):
                self.skipped_steps += 1
                self.flat_grad.zero_()
                self.micro = 0
                return
        self.step_count += 1
        for p, m1, m2 in zip(self.params, self.exp_avg, self.exp_avg_sq):
            tops.adam_step(p.data, p.grad, m1, m2, self.step_count, self.lr, self.betas, self.eps, grad_scale=coef)
            # adam_step writes through a raw pointer, which torch does not see: bump the parameter's version so
            # every cache keyed on it (fp16x2 pre-split ops.weight_split, W^T ptv3_train.wt) is rebuilt
            torch.autograd.graph.increment_version(p)
        self.flat_grad.zero_()
        self.micro = 0

    def state_dict(self) -> dict:
        """Optimiser state for a resume: Adam moments, step counts and the DropPath mask counter (so a resumed
        run draws new masks instead of replaying step 0's)."""
        return {"exp_avg": [t.detach().cpu() for t in self.exp_avg],
                "exp_avg_sq": [t.detach().cpu() for t in self.exp_avg_sq],
                "step_count": self.step_count, "skipped_steps": self.skipped_steps,
                "masks": self.masks.state_dict() if hasattr(self.masks, "state_dict") else None}

    def load_state_dict(self, sd: dict) -> None:
        for dst, src in zip(self.exp_avg + self.exp_avg_sq, list(sd["exp_avg"]) + list(sd["exp_avg_sq"])):
            dst.copy_(src)
        self.step_count = int(sd["step_count"])
        self.skipped_steps = int(sd.get("skipped_steps", 0))
        if sd.get("masks") is not None and hasattr(self.masks, "load_state_dict"):
            self.masks.load_state_dict(sd["masks"])

    def step(self, scenes, cameras, images, masks=None, perms=None) -> float:
        loss = self.micro_step(scenes, cameras, images, masks=masks, perms=perms)
        if self.micro % self.accumulate_step == 0:
            self.optimizer_step()
        return loss
