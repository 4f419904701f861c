"""FeaturePredictor on MI355X (mirror of reference models/feature_predictor.py:24-245).

Same constructor arguments (ptv3_base.gin values as defaults), same
submodules (`backbone` = PointTransformerV3Model, `features_outputhead` =
ModuleDict of Sequential(Linear, ReLU, ..., Linear)) and state-dict keys,
same `forward(batch_normalized_gs, batch_scene_idx) -> [refined gs dict]`.

Device path per scene (all libsfx HIP kernels):
  sfx_gs_pack      batchify feat [N,Cin] straight into the head input buffer
                   H0 = [y | feat] ([N, 96+Cin], row stride padded to 4)
                   + grid_coord = floor(coord*384) + grid max (depth)
  PTv3 backbone    writes its final [N,96] feature into H0[:, :96]
  heads            one GEMM for all six first layers (Cin_h -> 6*128, ReLU),
                   two grouped GEMMs (6 x 128x128, ReLU), one block-diagonal
                   GEMM to the 23 packed outputs with tanh on the means
                   columns and the residual (input attributes) fused
The refined Gaussians come back as views into one packed [N, 23] record,
which the fused render prep (sfx_render_prep_project) reads in place.
"""
from __future__ import annotations

import os
from collections import OrderedDict
from typing import Dict, List, Optional

import torch
import torch.nn as nn
from torch import Tensor

from . import _lib
from . import ptv3_ops as ops
from .ptv3 import PointTransformerV3Model

# renumber the points by serialized order inside the backbone (ptv3.PointTransformerV3.prepare): opt-in
# (SFX_REORDER=1), measured neutral on config B (profiles/r05_ab_reorder.txt)
REORDER = os.environ.get("SFX_REORDER", "0") == "1"
FEATURE2CHANNEL = {"means": 3, "features_dc": 3, "features_rest": 3, "opacities": 1, "scales": 3, "quats": 4}
ALL_FEATURES = ["means", "features_dc", "features_rest", "opacities", "scales", "quats"]
BASE_FEATURES = ["means", "scales", "opacities", "quats", "features_dc", "features_rest"]


def _channels(sh_degree):
    d = dict(FEATURE2CHANNEL)
    d["features_rest"] = ((sh_degree + 1) ** 2 - 1) * 3
    return d


class FeaturePredictor(nn.Module):
    def __init__(self, backbone_type="PT", sh_degree=1, input_features=BASE_FEATURES, input_feat_to_mlp=True,
                 output_features=BASE_FEATURES, output_head_nlayer=4, output_head_type="mlp-relu",
                 output_head_width=128, output_features_type="res", res_feature_activation=None,
                 max_scale_normalized=1e-2, grid_resolution=384, resume_ckpt=None, input_embed_to_mlp=False,
                 zeroinit=True, additional_info=None, backbone_kwargs: Optional[dict] = None):
        super().__init__()
        if backbone_type != "PT":
            raise NotImplementedError("backbone_type 'SP' (SparseUNet) is out of scope (SURVEY.md §2)")
        if output_head_type != "mlp-relu" or output_features_type != "res" or not input_feat_to_mlp:
            raise NotImplementedError("only the ptv3_base.gin head configuration is on the path")
        ch = _channels(sh_degree)
        self.sh_degree = sh_degree
        self.input_features = [f for f in input_features if not (f == "features_rest" and sh_degree == 0)]
        self.output_features = [f for f in output_features if not (f == "features_rest" and sh_degree == 0)]
        if self.input_features != [f for f in BASE_FEATURES if f in self.input_features]:
            raise NotImplementedError("input_features must follow ptv3_base.gin order")
        if self.output_features != self.input_features:
            raise NotImplementedError("output_features must equal input_features (ptv3_base.gin)")
        self.ch = ch
        in_channels = sum(ch[f] for f in self.input_features)
        self.gs_features_dim = in_channels
        self.grid_resolution = grid_resolution
        self.max_scale_normalized = max_scale_normalized
        self.output_features_type = output_features_type
        self.additional_info = additional_info or {}
        self.res_activation = {f: "tanh" if f == "means" else "identity" for f in self.output_features}
        if res_feature_activation is not None:
            for f, a in res_feature_activation.items():
                nm = type(a).__name__.lower() if not isinstance(a, str) else a.lower()
                self.res_activation[f] = "tanh" if "tanh" in nm else "identity"
            if any(self.res_activation[f] != ("tanh" if f == "means" else "identity") for f in self.output_features):
                raise NotImplementedError("res_feature_activation must be Tanh(means), Identity(others)")
        self.backbone = PointTransformerV3Model(in_channels=in_channels, additional_info=additional_info,
                                                **(backbone_kwargs or {}))
        head_in = self.backbone.output_dim + in_channels
        self.head_in = head_in
        self.nlayer = output_head_nlayer
        self.width = output_head_width
        self.features_outputhead = nn.ModuleDict()
        for f in self.output_features:
            layers = []
            for i in range(output_head_nlayer - 1):
                layers += [nn.Linear(head_in if i == 0 else output_head_width, output_head_width), nn.ReLU()]
            layers.append(nn.Linear(output_head_width if output_head_nlayer > 1 else head_in, ch[f]))
            self.features_outputhead[f] = nn.Sequential(*layers)
        if zeroinit:
            for m in self.features_outputhead.values():
                m[-1].weight.data.zero_()
                m[-1].bias.data.zero_()
        if resume_ckpt is not None:
            load_checkpoint(self, resume_ckpt)
        self._pack_cache = None

    # ---- packed head weights (rebuilt only when a parameter changes) --------------
    def _packed_heads(self):
        params = self.__dict__.get("_head_params")
        if params is None:  # (the heads' module structure is fixed; the list is built once)
            params = [p for f in self.output_features for p in self.features_outputhead[f].parameters()]
            self.__dict__["_head_params"] = params
        key = tuple((p.data_ptr(), p._version) for p in params)
        if self._pack_cache is not None and self._pack_cache[0] == key:
            return self._pack_cache[1]
        feats = self.output_features
        G, Wd = len(feats), self.width
        nl = self.nlayer
        heads = [self.features_outputhead[f] for f in feats]
        kpad = (self.head_in + 3) // 4 * 4  # pad K to a multiple of 4 -> vectorised GEMM loads
        with torch.no_grad():
            w1 = torch.nn.functional.pad(torch.cat([h[0].weight for h in heads], 0),
                                         (0, kpad - self.head_in)).contiguous()    # [G*128, kpad]
            b1 = torch.cat([h[0].bias for h in heads], 0).contiguous()
            mids = []
            for li in range(1, nl - 1):
                wm = torch.stack([h[2 * li].weight for h in heads], 0).contiguous()  # [G,128,128]
                bm = torch.stack([h[2 * li].bias for h in heads], 0).contiguous()
                mids.append((wm, bm))
            out_dim = sum(self.ch[f] for f in feats)
            wl = torch.zeros(out_dim, G * Wd, device=w1.device)
            bl = torch.zeros(out_dim, device=w1.device)
            r = 0
            for g, (f, h) in enumerate(zip(feats, heads)):
                c = self.ch[f]
                wl[r:r + c, g * Wd:(g + 1) * Wd] = h[-1].weight
                bl[r:r + c] = h[-1].bias
                r += c
        packed = (w1, b1, mids, wl.contiguous(), bl.contiguous(), out_dim)
        self._pack_cache = (key, packed)
        return packed

    @torch.no_grad()
    def refine_packed(self, gs: Dict[str, Tensor], perms=None) -> Tensor:
        """One scene -> packed refined record [N, Cin] (input_features layout)."""
        means = gs["means"]
        _lib.require_gpu(means)
        dev = means.device
        n = means.shape[0]
        cin = self.gs_features_dim
        cb = self.backbone.output_dim
        ld = (cb + cin + 3) // 4 * 4
        n_tanh = self.ch["means"] if self.output_features[0] == "means" else 0
        fused_heads = ops.heads_fused_ok(len(self.output_features), self.nlayer, self.width, self.head_in,
                                         sum(self.ch[f] for f in self.output_features))
        # the heads' pack check (a version key over every head parameter) runs here, while the GPU still
        # renders the previous scene, not between the backbone's last launch and the heads' (a host gap)
        heads_pack = self._fused_heads() if fused_heads else None
        h0 = torch.zeros(n, ld, device=dev, dtype=torch.float32)
        feat = h0[:, cb:cb + cin]
        grid = torch.empty(n, 3, device=dev, dtype=torch.int32)
        gmax = torch.zeros(1, device=dev, dtype=torch.int32)
        ops.gs_pack(gs, feat, float(self.grid_resolution), grid, gmax)
        # Pointcept: int(grid_coord.max()).bit_length(), read back asynchronously (the backbone's embedding
        # GEMM runs while the host waits for it)
        data = {"coord": means, "grid_coord": grid, "offset": [n], "feat": feat,
                "serialized_depth": _lib.HostRead(gmax)}
        method = self.additional_info.get("downsample")
        if method is None:
            # REORDER: the backbone runs on the points renumbered by serialized order and writes its features
            # back in input order (result-neutral)
            self.backbone(data, perms=perms, out=h0[:, :cb], reorder=REORDER)
        else:  # fork experiment (feature_predictor.py:159-196): backbone on the downsampled cloud, mapped back
            from .downsample import downsample_for_backbone
            c, f, g, mapper = downsample_for_backbone(method, self.additional_info, means, feat, grid)
            y = self.backbone({"coord": c, "grid_coord": g, "offset": [c.shape[0]], "feat": f}, perms=perms).feat
            h0[:, :cb] = mapper(y)
        if heads_pack is not None:
            st, pr, ocols, out_dim = heads_pack
            # all six heads + tanh + residual in one launch (csrc/heads.hip): no [N, 768] hidden in HBM
            return ops.heads(h0, self.head_in, cb, out_dim, n_tanh, ocols, st, pr)
        w1, b1, mids, wl, bl, out_dim = self._packed_heads()
        x = h0[:, :w1.shape[1]]  # [y | feat | 0-pad]
        h = ops.linear(x, w1, b1, act=ops.ACT_RELU)
        for wm, bm in mids:
            h = ops.grouped_linear(h, wm, bm, len(self.output_features), act=ops.ACT_RELU)
        return ops.linear(h, wl, bl, act=ops.ACT_TANH, act_ncols=n_tanh, residual=feat)

    def check_refine(self, wait: bool = True) -> None:
        """Validate the pooled run counts of the refines issued so far (PointTransformerV3.check_deferred): call
        where a refined result is consumed on the host (evaluate_scenes does, at its metric readback).  Raises once
        per failing forward, naming it; the model stays usable.  With `wait`, also the stream's look-back scans
        (serialization / pooling / intersection sorts: _lib.check_lookback; the stream is drained there)."""
        self.backbone.backbone.check_deferred(wait=wait)
        if wait:
            _lib.check_lookback("FeaturePredictor.check_refine")

    def _fused_heads(self):
        """(slab stream, parameter table, output columns, out_dim) of the fused heads kernel, rebuilt with the
        packed heads (when a head parameter changes)."""
        packed = self._packed_heads()
        cache = self.__dict__.get("_fused_heads_cache")
        if cache is None or cache[0] is not packed:
            w1, b1, mids, wl, bl, out_dim = packed
            ocols = [0]
            for f in self.output_features:
                ocols.append(ocols[-1] + self.ch[f])
            with torch.no_grad():
                st, pr, keep = ops.heads_pack(w1, b1, mids, wl, bl, len(self.output_features), self.head_in, ocols)
            cache = (packed, st, pr, ocols, out_dim, keep)
            self.__dict__["_fused_heads_cache"] = cache
        return cache[1], cache[2], cache[3], cache[4]

    def unpack(self, packed: Tensor) -> Dict[str, Tensor]:
        out = OrderedDict()
        c = 0
        for f in self.output_features:
            w = self.ch[f]
            v = packed[:, c:c + w]
            if f == "features_rest":
                v = v.view(packed.shape[0], -1, 3) if v.is_contiguous() else v.unflatten(1, (-1, 3))
            out[f] = v
            c += w
        return out

    def forward(self, batch_normalized_gs: List[Dict[str, Tensor]], batch_scene_idx: List, perms=None, **kwargs):
        outs = []
        for gs in batch_normalized_gs:
            packed = self.refine_packed(gs, perms=perms)
            o = self.unpack(packed)
            for key in ALL_FEATURES:
                if self.sh_degree == 0 and key == "features_rest":
                    continue
                if key not in o:
                    o[key] = gs[key]
            outs.append(o)
        assert len(outs) == 1, "Now only support batch size 1"
        return outs


def convert_state_dict(sd: Dict[str, Tensor], target: Dict[str, Tensor]) -> Dict[str, Tensor]:
    """A checkpoint of the reference FeaturePredictor (train.py:344 saves `model.module.state_dict()` after the
    SyncBatchNorm conversion of train.py:404) -> this module's state dict.

    * a DDP `module.` prefix is stripped (checkpoints saved without `.module`);
    * SyncBatchNorm and BatchNorm1d share their keys (weight, bias, running_mean, running_var,
      num_batches_tracked) -- nothing to convert;
    * SubMConv3d weights: spconv 2.x stores [Cout, 3, 3, 3, Cin] (this layout); an spconv 1.x checkpoint's
      [3, 3, 3, Cin, Cout] is permuted to it.  (Which (x, y, z) neighbour each of the 27 kernel taps reads
      follows Pointcept's spconv call; the tap order itself is parity unpinned)
    """
    if sd and all(k.startswith("module.") for k in sd):
        sd = {k[len("module."):]: v for k, v in sd.items()}
    out = {}
    for k, v in sd.items():
        t = target.get(k)
        if t is not None and v.dim() == 5 and tuple(v.shape) != tuple(t.shape):
            if tuple(v.permute(4, 0, 1, 2, 3).shape) == tuple(t.shape):
                v = v.permute(4, 0, 1, 2, 3).contiguous()
        out[k] = v
    return out


def load_checkpoint(model: nn.Module, ckpt, strict: bool = True):
    """Load a reference checkpoint (path or state dict; `torch.load(weights_only=True)`, never unpickling
    arbitrary objects) into `model` through convert_state_dict.  Cached derived weights (folded CPE convs,
    packed heads) are keyed on the parameters' versions, so they are rebuilt on the next forward."""
    sd = torch.load(ckpt, map_location="cpu", weights_only=True) if isinstance(ckpt, (str, bytes)) else ckpt
    if isinstance(sd, dict) and "state_dict" in sd and isinstance(sd["state_dict"], dict):
        sd = sd["state_dict"]
    return model.load_state_dict(convert_state_dict(sd, model.state_dict()), strict=strict)

