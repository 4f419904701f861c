"""Device ops of the PTv3 refiner: thin typed wrappers over the libsfx C-ABI.

Every function allocates its outputs with torch (device memory plumbing) and
launches HIP kernels on the current stream.  No torch compute ops and no CPU
fallback: a missing library or a CPU tensor raises.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
from torch import Tensor

from . import _lib
from ._lib import I, L, P, F, Z, call, ptr, stream

_lib.register("sfx_linear", [I, I, I, P, L, P, I, P, L, P, P, P, I, I, P, L, P, P, L, P, L, I, L, L, L, L, P, P, I,
                              P, I, P, I, P, I, P, P, P])
_lib.register("sfx_weight_split", [I, I, P, L, P, P, P])
_lib.register("sfx_amax_f32", [I, I, P, L, P, I, P])
_lib.register("sfx_ln_amax_bound", [I, P, P, P, I, P])
_lib.register("sfx_layernorm", [I, I, P, L, P, P, F, P, L, P])
_lib.register("sfx_cpe_residual_ln", [I, I, P, P, P, P, P, P, F, P, P, P])
_lib.register("sfx_cpe_residual_ln_pairs", [I, I, P, L, P, P, L, P, P, P, P, P, F, P, P, P])
_lib.register("sfx_cpe_ln_qkv_pairs", [I, I, P, L, P, P, L, P, P, P, P, P, F, P, P, P, P, P, P, I, P])
_lib.register("sfx_window_attention", [I, I, I, I, I, P, P, P, F, P, P, I, P])
_lib.register("sfx_window_attention_varlen", [I, I, I, I, I, P, P, P, F, P, P, I, P])
_lib.register("sfx_window_attention_proj", [I, I, I, I, I, P, P, P, F, P, I, P, P, P, P, L, P, L, P])
_lib.register("sfx_serialize_keys", [I, P, P, I, I, I, I, I, I, I, P, P, P])
_lib.register("sfx_serialize_finalize", [I, I, P, P, P, P])
_lib.register("sfx_serialize_permute", [I, I, P, P, P, P, P, P, P, P, P, P, P])
_lib.register("sfx_pool_run_flags", [I, I, P, P, I, P, P])
_lib.register("sfx_pool_run_counts", [I, P, P, P, I, P, P])
_lib.register("sfx_pool_assign_runs", [I, I, I, P, P, P, P, P, P, P, P])
_lib.register("sfx_pool_reorder", [I, I, I, P, P, P, P, P, P, P])
_lib.register("sfx_pool_gather", [I, I, I, P, P, I, P, P, I, P, P, P, P, P])
_lib.register("sfx_segment_max_affine_act", [I, I, P, P, P, P, P, I, P, P])
_lib.register("sfx_segment_mean", [I, I, P, P, P, P, P])
_lib.register("sfx_subm_table_log2", [I])
_lib.register("sfx_subm_neighbors", [I, P, P, I, P, P, P, P, P, P])
_lib.register("sfx_subm_permute", [I, P, P, P, P, P, P])
_lib.register("sfx_subm_pairs_workspace_bytes", [I], Z)
_lib.register("sfx_subm_pairs", [I, P, P, Z, P, P, P, I, P])
_lib.register("sfx_subm_conv", [I, I, I, P, L, P, P, P, P, P, P, P, L, P, I, P, I, P, P, P])
_lib.register("sfx_subm_conv_partials", [I, I, I, P, L, P, P, P, P, P, P, P, L, P, L, P, P, P])
_lib.register("sfx_subm_conv_partials_pairs", [I, I, I, P, L, P, P, P, P, P, P, P, L, P, L, P, P, P])
_lib.register("sfx_subm_pair_pos", [I, L, P, P, P, P])
_lib.register("sfx_subm_pair_lists_workspace_bytes", [I], Z)
_lib.register("sfx_subm_pair_lists", [I, P, P, Z, P, P, P, P, P, I, P])
_lib.register("sfx_cpe_residual_ln_cpairs", [I, I, P, L, P, P, L, P, P, P, P, P, F, P, P, P])
_lib.register("sfx_subm_cpe_pack_bytes", [I], Z)
_lib.register("sfx_subm_cpe_pack", [I, P, P, P, P, P])
_lib.register("sfx_subm_cpe_ln", [I, I, P, P, P, P, P, P, P, P, P, P, P, P, F, P, P, P])
_lib.register("sfx_subm_order_keys", [I, P, P, P])
_lib.register("sfx_subm_rowexp", [I, I, P, P, P])
_lib.register("sfx_gs_pack", [I, P, L, P, L, P, L, P, L, P, L, P, L, I, F, P, L, P, P, P])
_lib.register("sfx_offsets_to_batch", [I, I, P, P, P])
_lib.register("sfx_move_rows", [L, I, P, L, P, P, L, I, P])
_lib.register("sfx_point_embed", [I, I, I, P, L, P, P, P, P, P, L, P])
_lib.register("sfx_heads_stream_floats", [I, I], Z)
_lib.register("sfx_heads_params_floats", [I], Z)
_lib.register("sfx_heads_pack", [I, I, I, P, I, P, P, P, P, P, P, P, P, P])
_lib.register("sfx_heads", [I, I, I, I, P, L, I, I, P, P, P, P, P])
_lib.register("sfx_gemm_force_config", [I, I])
_lib.register("sfx_set_precision", [I])
_lib.register("sfx_get_precision", [])
_lib.register("sfx_mlp_stream_floats", [I], Z)
_lib.register("sfx_mlp_params_floats", [I], Z)
_lib.register("sfx_mlp_pack", [I, P, P, P, P, P, P, P, P, P, P])
_lib.register("sfx_block_mlp", [I, I, P, L, P, P, F, P, L, P, P])
_lib.register("sfx_block_mlp_train", [I, I, P, L, P, P, F, P, P, P, L, P])
_lib.register("sfx_block_mlp_bwd", [I, I, P, L, P, P, P, P, P, L, P])

ACT_NONE, ACT_GELU, ACT_RELU, ACT_TANH = 0, 1, 2, 3
# gemm.hip kCfgs: 128x128, 128x96, 128x64, 64x128, 64x64 (4 waves, 2 per CU), 256x128, 128x256 (8 waves)
GEMM_NUM_CONFIGS = 7


def gemm_force_config(cfg: int = -1, stream_k: int = -1) -> None:
    """Tuning / test hook: force the GEMM tile configuration and Stream-K choice (-1 = cost model)."""
    call("sfx_gemm_force_config", cfg, stream_k)


# Library operand-precision modes (include/sfx.h sfx_set_precision): "fp32" = fp32-accurate split operands (the
# default), "amp" = reference precision, the class of the reference's fp16 autocast training (train.py:240,
# configs/train/default.gin:11 enable_amp): leading fp16 term product only in the GEMM family.
PRECISIONS = {"fp32": 0, "amp": 1}


def get_precision() -> str:
    m = _lib.fn("sfx_get_precision")()
    return {v: k for k, v in PRECISIONS.items()}[m]


@contextlib.contextmanager
def precision(mode: str):
    """Run the enclosed launches in precision `mode` ("fp32" | "amp"); restores the previous mode."""
    if mode not in PRECISIONS:
        raise ValueError(f"precision {mode!r}: expected one of {sorted(PRECISIONS)}")
    prev = _lib.fn("sfx_get_precision")()
    call("sfx_set_precision", PRECISIONS[mode])
    try:
        yield
    finally:
        call("sfx_set_precision", prev)
ORDER_TYPES = {"z": 0, "z-trans": 1, "hilbert": 2, "hilbert-trans": 3}


# ---- fp16x2 operand maxima ("amax slots", include/sfx.h) ----------------------------------------------------
# A slot is (device pointer to 64 u64 sub-slots, tag).  The GEMM scales its fp16x2 operands from upper bounds
# of their largest magnitudes: the refiner passes the slots its producers fill (GEMM epilogues, LayerNorm
# weight bounds, cached weight maxima); a GEMM without one runs the library's own maxima pass.
AMAX_SUB = 64
_AMAX_RING = 4096
_amax_state: dict = {}


def new_amax(device) -> Tuple[int, int]:
    """A fresh (slot pointer, tag) from a per-device ring (zero-initialised once; tags only grow)."""
    st = _amax_state.get(device)
    if st is None:
        buf = torch.zeros(_AMAX_RING * AMAX_SUB, dtype=torch.int64, device=device)
        st = _amax_state[device] = [buf, 0, 0]
    buf = st[0]
    st[1] = (st[1] + 1) % _AMAX_RING
    st[2] = st[2] + 1 if st[2] < 0x7FFFFFFF else 1
    return buf.data_ptr() + 8 * AMAX_SUB * st[1], st[2]


def _own_slot(device) -> Tuple[Tensor, Tuple[int, int]]:
    """A dedicated, never-recycled amax slot (its own zeroed 64-u64 buffer, tag 1) for a cached bound: the ring
    of `new_amax` wraps every _AMAX_RING launches, after which a later producer would overwrite a cached slot."""
    buf = torch.zeros(AMAX_SUB, dtype=torch.int64, device=device)
    return buf, (buf.data_ptr(), 1)


def weight_amax(w: Tensor) -> Tuple[int, int]:
    """max |W| of a weight matrix (2-D view), cached on the tensor (in its own slot) until its storage or version
    changes."""
    key = (w.data_ptr(), w._version, tuple(w.shape))
    c = getattr(w, "_sfx_wamax", None)
    if c is not None and c[0] == key:
        return c[2]
    w2 = w.reshape(w.shape[0], -1)
    buf, slot = _own_slot(w.device)
    call("sfx_amax_f32", w2.shape[0], w2.shape[1], ptr(w2), w2.stride(0), slot[0], slot[1], stream())
    w._sfx_wamax = (key, buf, slot)
    return slot


def ln_amax(gamma: Tensor, beta: Tensor) -> Tuple[int, int]:
    """Bound sqrt(C-1) max|gamma| + max|beta| of a LayerNorm's outputs, cached on gamma (in its own slot)."""
    key = (gamma.data_ptr(), gamma._version, beta.data_ptr(), beta._version)
    c = getattr(gamma, "_sfx_lnamax", None)
    if c is not None and c[0] == key:
        return c[2]
    buf, slot = _own_slot(gamma.device)
    call("sfx_ln_amax_bound", gamma.shape[0], ptr(gamma), ptr(beta), slot[0], slot[1], stream())
    gamma._sfx_lnamax = (key, buf, slot)
    return slot


SPLIT_MIN_K = 64  # K below which the GEMM runs exact fp32 MFMA (gemm.hip split_mode)


def weight_split(w: Tensor, rows: Optional[int] = None) -> Tuple[Optional[int], Optional[int]]:
    """(split, 1/scale) device pointers of the fp16x2 pre-split of a weight viewed as [rows, cols] (default
    rows = w.shape[0]; sfx_weight_split, include/sfx.h), cached on the tensor until its storage or version
    changes.  (None, None) when the GEMM would not use it (cols < 64 or not a multiple of 4)."""
    rows = w.shape[0] if rows is None else rows
    cols = w.numel() // rows
    if cols < SPLIT_MIN_K or cols % 4:
        return None, None
    key = (w.data_ptr(), w._version, tuple(w.shape), rows)
    c = getattr(w, "_sfx_wsplit", None)
    if c is not None and c[0] == key:
        return c[1].data_ptr(), c[2].data_ptr()
    w2 = w.reshape(rows, cols)
    if w2.stride(1) != 1 or w2.stride(0) % 4 or w2.data_ptr() % 16:
        w2 = w2.contiguous()
    sp = torch.empty(rows, cols, device=w.device, dtype=torch.float32)
    inv = torch.empty(rows, device=w.device, dtype=torch.float32)
    call("sfx_weight_split", rows, cols, ptr(w2), w2.stride(0), ptr(sp), ptr(inv), stream())
    w._sfx_wsplit = (key, sp, inv)
    return sp.data_ptr(), inv.data_ptr()


def _slot_args(slot: Optional[Tuple[int, int]]):
    return (None, 0) if slot is None else slot


def _rows(t: Tensor) -> Tuple[int, int]:
    """(pointer, leading dimension) of a 2-D row-major (possibly column-sliced) float32 matrix."""
    if t.dim() != 2 or t.stride(1) != 1:
        raise RuntimeError("expected a 2-D tensor with unit column stride")
    if not t.is_cuda:
        raise RuntimeError("expected a device tensor")
    if t.dtype != torch.float32:
        raise RuntimeError(f"expected float32, got {t.dtype}")
    return t.data_ptr(), t.stride(0)


def linear(x: Tensor, weight: Tensor, bias: Optional[Tensor] = None, *, act: int = ACT_NONE, act_ncols: int = -1,
           scale: Optional[Tensor] = None, shift: Optional[Tensor] = None, residual: Optional[Tensor] = None,
           residual_idx: Optional[Tensor] = None, out: Optional[Tensor] = None, pre_out: Optional[Tensor] = None,
           gather_idx: Optional[Tensor] = None, rows: Optional[int] = None,
           out_rows: Optional[Tensor] = None, rowscale: Optional[Tensor] = None,
           pre_before_act: bool = False, a_amax: Optional[Tuple[int, int]] = None,
           w_amax: Optional[Tuple[int, int]] = None, y_amax: bool = False):
    """y = act((x W^T + b) * scale + shift) + residual[residual_idx]  (csrc/gemm.hip: fp32-accurate MFMA GEMM,
    fp16x2 split operands for K >= 64, exact f32 MFMA below; SFX_GEMM_PREC=bf16x3|fp32 select the others).

    a_amax / w_amax: amax slots bounding |x| / |W| (None: the library measures them); y_amax=True returns
    (y, slot of max |y|) for the consumer of y.

    With `gather_idx` [M, S] (int32, -1 = empty) the A operand is the implicit
    concatenation of S gathered rows of `x` (SubMConv3d as implicit GEMM).
    Training forward: `rowscale` multiplies each row's branch value before the residual add (DropPath),
    `pre_out` + `pre_before_act` saves the pre-activation for the backward."""
    N, K = weight.shape
    if gather_idx is not None:
        M = gather_idx.shape[0]
        S = gather_idx.shape[1]
        if K != S * x.shape[1]:
            raise RuntimeError("gathered linear: weight K must be segments * x.shape[1]")
    else:
        M = x.shape[0] if rows is None else rows
        S = 1
        if x.shape[1] != K:
            raise RuntimeError(f"linear: x has {x.shape[1]} features, weight expects {K}")
    if out is None:
        out = torch.empty(M, N, device=weight.device, dtype=torch.float32)
    pa, lda = _rows(x)
    pw, ldw = _rows(weight)
    py, ldy = _rows(out)
    pr, ldr = _rows(residual) if residual is not None else (None, 0)
    pp, ldp = _rows(pre_out) if pre_out is not None else (None, 0)
    ys = new_amax(out.device) if y_amax else None
    call("sfx_linear", M, N, K, pa, lda, ptr(gather_idx), S, pw, ldw, ptr(bias), ptr(scale), ptr(shift), act,
         act_ncols, pr, ldr, ptr(residual_idx), py, ldy, pp, ldp, 1, 0, 0, 0, 0, ptr(out_rows), ptr(rowscale),
         1 if pre_before_act else 0, *_slot_args(a_amax), *_slot_args(w_amax), *_slot_args(ys),
         *weight_split(weight), stream())
    return (out, ys) if y_amax else out


def point_embed_ok(x: Tensor, weight: Tensor) -> bool:
    N, K = weight.shape
    return K <= 64 and N in (32, 64) and x.dim() == 2 and x.stride(1) == 1


def point_embed(x: Tensor, weight: Tensor, bias: Optional[Tensor], scale: Optional[Tensor],
                shift: Optional[Tensor]) -> Tensor:
    """GELU((x W^T + b) * scale + shift) for K <= 64 inputs (the PTv3 embedding, pointtransformer_v3.py:273-278):
    one fp32-VALU launch (csrc/misc.hip) instead of a K < 64 GEMM tile."""
    N, K = weight.shape
    M = x.shape[0]
    out = torch.empty(M, N, device=x.device, dtype=torch.float32)
    px, ldx = _rows(x)
    call("sfx_point_embed", M, K, N, px, ldx, ptr(weight.detach().contiguous()), ptr(bias), ptr(scale), ptr(shift),
         ptr(out), N, stream())
    return out


# FeaturePredictor heads in one launch (csrc/heads.hip); SFX_HEADS_FUSED=0: the four GEMM launches
HEADS_FUSED = os.environ.get("SFX_HEADS_FUSED", "1") != "0"


def heads_fused_ok(ng: int, nlayer: int, width: int, kin: int, out_dim: int) -> bool:
    return HEADS_FUSED and nlayer == 4 and width == 128 and 1 <= ng <= 6 and kin <= 160 and out_dim <= 64


def heads_pack(w1: Tensor, b1: Tensor, mids, wl: Tensor, bl: Tensor, ng: int, kin: int, ocols: List[int]):
    """Packed head weights (FeaturePredictor._packed_heads layout) -> (fp16x2 slab stream, parameter table) of
    sfx_heads: w1 [ng*128, >=kin], mids = [(wm [ng,128,128], bm [ng,128])] x 2, wl [out_dim, ng*128] block
    diagonal, bl [out_dim]."""
    dev = w1.device
    out_dim = wl.shape[0]
    wm = torch.stack([m[0] for m in mids], 0).contiguous()
    bm = torch.stack([m[1] for m in mids], 0).contiguous()
    w4 = torch.empty(out_dim, 128, device=dev, dtype=torch.float32)
    for g in range(ng):
        w4[ocols[g]:ocols[g + 1]] = wl[ocols[g]:ocols[g + 1], g * 128:(g + 1) * 128]
    st = torch.empty(int(_lib.fn("sfx_heads_stream_floats")(ng, kin)), device=dev, dtype=torch.float32)
    pr = torch.empty(int(_lib.fn("sfx_heads_params_floats")(out_dim)), device=dev, dtype=torch.float32)
    ws = torch.empty(3 * ng * 128, device=dev, dtype=torch.int32)
    w1c = w1.contiguous()
    call("sfx_heads_pack", ng, kin, out_dim, ptr(w1c), w1c.shape[1], ptr(b1.contiguous()), ptr(wm), ptr(bm), ptr(w4),
         ptr(bl.contiguous()), ptr(st), ptr(pr), ptr(ws), stream())
    return st, pr, (w1c, wm, bm, w4)


def heads(x: Tensor, kin: int, res_off: int, out_dim: int, n_tanh: int, ocols: List[int], st: Tensor,
          pr: Tensor) -> Tensor:
    """y [N, out_dim] = heads(x[:, :kin]) + x[:, res_off:res_off+out_dim] (tanh on the first n_tanh columns)."""
    M = x.shape[0]
    px, ldx = _rows(x)
    y = torch.empty(M, out_dim, device=x.device, dtype=torch.float32)
    oc = (ctypes.c_int * len(ocols))(*ocols)
    call("sfx_heads", M, len(ocols) - 1, kin, out_dim, px, ldx, res_off, n_tanh, oc, ptr(st), ptr(pr), ptr(y),
         stream())
    return y


def grouped_linear(x: Tensor, weight: Tensor, bias: Tensor, groups: int, *, act: int = ACT_NONE,
                   out: Optional[Tensor] = None, a_amax: Optional[Tuple[int, int]] = None,
                   w_amax: Optional[Tuple[int, int]] = None, y_amax: bool = False):
    """Block-diagonal linear: x [M, G*K] -> [M, G*N] with weight [G, N, K], bias [G, N] (one launch);
    amax slots as in `linear`."""
    G, N, K = weight.shape
    M = x.shape[0]
    if out is None:
        out = torch.empty(M, G * N, device=x.device, dtype=torch.float32)
    pa, lda = _rows(x)
    py, ldy = _rows(out)
    ys = new_amax(out.device) if y_amax else None
    call("sfx_linear", M, N, K, pa, lda, None, 1, ptr(weight), K, ptr(bias), None, None, act, -1, None, 0, None, py,
         ldy, None, 0, G, K, N * K, N, N, None, None, 0, *_slot_args(a_amax), *_slot_args(w_amax),
         *_slot_args(ys), *weight_split(weight, G * N), stream())
    return (out, ys) if y_amax else out


# ---- fused Block MLP tail (csrc/mlp.hip) ---------------------------------------------------------------------
MLP_FUSED = os.environ.get("SFX_MLP_FUSED", "1") != "0"  # SFX_MLP_FUSED=0: LayerNorm + two GEMM launches
MLP_CHANNELS = (64, 96, 128, 256)  # what sfx_block_mlp serves
# where the eval forward uses it: every channel count it serves -- with the round-4 GELU it is 1.12-1.68x faster
# than LayerNorm + two GEMMs, C = 256 included (230.9 vs 259.2 us; round 3: 0.92x there, profiles/r03_mlp_bench.txt);
# SFX_MLP_CHANNELS=64,96,128 restores round 3's choice
MLP_FUSED_CHANNELS = tuple(int(c) for c in os.environ.get("SFX_MLP_CHANNELS", "64,96,128,256").split(",") if c)


def mlp_pack(ln2, fc1, fc2) -> Tuple[Tensor, Tensor]:
    """(weight stream, parameter table) of sfx_block_mlp for LayerNorm `ln2` and Linear `fc1` / `fc2`: the fp16x2
    pre-split W1 / W2 laid out as the kernel's LDS-DMA slabs, plus gamma / beta / biases / row scales.  Cached on
    fc1 until one of the six tensors changes (storage or version)."""
    ts = (ln2.weight, ln2.bias, fc1.weight, fc1.bias, fc2.weight, fc2.bias)
    key = tuple((t.data_ptr(), t._version) for t in ts)
    c = fc1.__dict__.get("_sfx_mlp")
    if c is not None and c[0] == key:
        return c[1], c[2]
    C = fc1.weight.shape[1]
    dev = fc1.weight.device
    st = torch.empty(int(_lib.fn("sfx_mlp_stream_floats")(C)), device=dev, dtype=torch.float32)
    pr = torch.empty(int(_lib.fn("sfx_mlp_params_floats")(C)), device=dev, dtype=torch.float32)
    ws = torch.empty(9 * C, device=dev, dtype=torch.int32)
    w = [t.detach().contiguous() for t in ts]
    call("sfx_mlp_pack", C, ptr(w[2]), ptr(w[3]), ptr(w[4]), ptr(w[5]), ptr(w[0]), ptr(w[1]), ptr(st), ptr(pr),
         ptr(ws), stream())
    fc1.__dict__["_sfx_mlp"] = (key, st, pr, w)
    return st, pr


def block_mlp_ok(x: Tensor, C: int) -> bool:
    return MLP_FUSED and C in MLP_FUSED_CHANNELS and C in MLP_CHANNELS and x.dim() == 2 and x.stride(1) == 1 and x.data_ptr() % 16 == 0 \
        and x.stride(0) % 4 == 0


def block_mlp(x2: Tensor, ln2, fc1, fc2, out: Optional[Tensor] = None, rowexp: Optional[Tensor] = None) -> Tensor:
    """Y = x2 + fc2(GELU(fc1(LN2(x2)))) in one launch (Block.forward's norm2 / mlp / shortcut, calflops.py:72-82;
    csrc/mlp.hip): the LayerNorm output and the [M, 4C] hidden stay on chip.  C in MLP_CHANNELS."""
    M, C = x2.shape
    st, pr = mlp_pack(ln2, fc1, fc2)
    if out is None:
        out = torch.empty(M, C, device=x2.device, dtype=torch.float32)
    px, ldx = _rows(x2)
    py, ldy = _rows(out)
    call("sfx_block_mlp", M, C, px, ldx, ptr(st), ptr(pr), float(ln2.eps), py, ldy, ptr(rowexp, torch.int32), stream())
    return out


def block_mlp_train(x2: Tensor, ln2, fc1, fc2, z: Tensor, rowscale: Optional[Tensor] = None,
                    out: Optional[Tensor] = None) -> Tensor:
    """Training forward of the Block MLP tail in one launch (csrc/mlp.hip MLP_TRAIN): Y = x2 + rowscale *
    (fc2(GELU(z)) + b2) with z = fc1(LN2(x2)) stored into `z` [M, 4C] for the backward."""
    M, C = x2.shape
    if z.shape != (M, 4 * C) or not z.is_contiguous():
        raise ValueError("block_mlp_train: z must be a contiguous [M, 4C] tensor")
    st, pr = mlp_pack(ln2, fc1, fc2)
    if out is None:
        out = torch.empty(M, C, device=x2.device, dtype=torch.float32)
    px, ldx = _rows(x2)
    py, ldy = _rows(out)
    call("sfx_block_mlp_train", M, C, px, ldx, ptr(st), ptr(pr), float(ln2.eps), ptr(rowscale), ptr(z), py, ldy,
         stream())
    return out


def mlp_bwd_pack(ln2, fc1, fc2) -> Tuple[Tensor, Tensor]:
    """sfx_block_mlp_bwd's weight stream / table: sfx_mlp_pack of W2^T in fc1's place and W1^T in fc2's, zero
    biases; cached on fc2 until a weight changes."""
    ts = (fc1.weight, fc2.weight)
    key = tuple((t.data_ptr(), t._version) for t in ts)
    c = fc2.__dict__.get("_sfx_mlp_bwd")
    if c is not None and c[0] == key:
        return c[1], c[2]
    C = fc1.weight.shape[1]
    dev = fc1.weight.device
    st = torch.empty(int(_lib.fn("sfx_mlp_stream_floats")(C)), device=dev, dtype=torch.float32)
    pr = torch.empty(int(_lib.fn("sfx_mlp_params_floats")(C)), device=dev, dtype=torch.float32)
    ws = torch.empty(9 * C, device=dev, dtype=torch.int32)
    w1t = fc2.weight.detach().t().contiguous()  # [4C, C]: rows = hidden units (W2^T)
    w2t = fc1.weight.detach().t().contiguous()  # [C, 4C]: rows = channels (W1^T)
    z4, z1 = torch.zeros(4 * C, device=dev), torch.zeros(C, device=dev)
    one = torch.ones(C, device=dev)
    call("sfx_mlp_pack", C, ptr(w1t), ptr(z4), ptr(w2t), ptr(z1), ptr(one), ptr(z1), ptr(st), ptr(pr), ptr(ws),
         stream())
    fc2.__dict__["_sfx_mlp_bwd"] = (key, st, pr, (w1t, w2t, z4, z1, one))
    return st, pr


def block_mlp_bwd(dy: Tensor, ln2, fc1, fc2, z: Tensor, rowscale: Optional[Tensor] = None,
                  out: Optional[Tensor] = None) -> Tensor:
    """d(LN2 output) of the Block MLP branch in one launch (csrc/mlp.hip MLP_BWD): W1^T (GELU'(z) o W2^T
    (rowscale * dy)) -- the [M, 4C] hidden gradient never reaches HBM."""
    M, C = dy.shape
    if z.shape != (M, 4 * C) or not z.is_contiguous():
        raise ValueError("block_mlp_bwd: z must be a contiguous [M, 4C] tensor")
    st, pr = mlp_bwd_pack(ln2, fc1, fc2)
    if out is None:
        out = torch.empty(M, C, device=dy.device, dtype=torch.float32)
    pd, ldd = _rows(dy)
    po, ldo = _rows(out)
    call("sfx_block_mlp_bwd", M, C, pd, ldd, ptr(st), ptr(pr), ptr(rowscale), ptr(z), po, ldo, stream())
    return out


def layernorm(x: Tensor, gamma: Tensor, beta: Tensor, eps: float, out: Optional[Tensor] = None) -> Tensor:
    M, C = x.shape
    if out is None:
        out = torch.empty(M, C, device=x.device, dtype=torch.float32)
    px, ldx = _rows(x)
    py, ldy = _rows(out)
    call("sfx_layernorm", M, C, px, ldx, ptr(gamma), ptr(beta), float(eps), py, ldy, stream())
    return out


def cpe_residual_ln(t, x: Tensor, g_cpe: Tensor, b_cpe: Tensor, g1: Tensor, b1: Tensor, eps: float,
                    x_out: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
    """x' = x + LN_cpe(t); h = LN_norm1(x')  (Block cpe tail + shortcut + norm1).  t is the conv output, or a
    `SubmPartials` (subm_conv(..., partials=True)): the centre output plus the pair partials, summed here per row in
    a fixed offset order."""
    M, C = x.shape
    x_out = torch.empty_like(x) if x_out is None else x_out
    h = torch.empty_like(x)
    if isinstance(t, SubmPartials):
        # compacted positions (fewer position / row loads; at C = 256 HBM-bound either way, 102.2 vs 100.6 us for the
        # [n][27] kernel, whose index the lists then need not write: profiles/r06_ab_ln_compact.txt)
        if t.cpos is not None:
            call("sfx_cpe_residual_ln_cpairs", M, C, ptr(t.centre), t.ldt, ptr(t.partials), ptr(t.cpos), t.num_pairs,
                 ptr(x), ptr(g_cpe), ptr(b_cpe), ptr(g1), ptr(b1), float(eps), ptr(x_out), ptr(h), stream())
        else:
            call("sfx_cpe_residual_ln_pairs", M, C, ptr(t.centre), t.ldt, ptr(t.partials), ptr(t.pair_pos),
                 t.num_pairs, ptr(x), ptr(g_cpe), ptr(b_cpe), ptr(g1), ptr(b1), float(eps), ptr(x_out), ptr(h), stream())
    else:
        call("sfx_cpe_residual_ln", M, C, ptr(t), ptr(x), ptr(g_cpe), ptr(b_cpe), ptr(g1), ptr(b1), float(eps),
             ptr(x_out), ptr(h), stream())
    return x_out, h


# the pair-sum CPE LayerNorm + norm1 + qkv projection as one launch on the eval Block (csrc/norm.hip
# cpe_ln_qkv_kernel, ABI v15).  Opt-in (SFX_LN_QKV=1): measured slower on config B (C = 128: 222 us vs 78 + 68 us for
# the LayerNorm launch + qkv GEMM; C = 96: 133 vs 58 + 54; C = 64: 77 vs 42 + 38; 602 vs 621 renders/s,
# profiles/r06_ab_ln_qkv.txt): 128-row workgroups at two per CU keep far fewer pair-partial gathers in flight than
# the LayerNorm kernel's 8-row workgroups, and the LayerNorm phase is the latency-bound part
LN_QKV = os.environ.get("SFX_LN_QKV", "0") == "1"
LN_QKV_CHANNELS = (64, 96, 128)


def cpe_ln_qkv_ok(t, C: int, qkv_weight: Tensor) -> bool:
    return (LN_QKV and isinstance(t, SubmPartials) and C in LN_QKV_CHANNELS and get_precision() == "fp32"
            and weight_split(qkv_weight)[0] is not None)


def cpe_ln_qkv(t: "SubmPartials", x: Tensor, g_cpe: Tensor, b_cpe: Tensor, g1: Tensor, b1: Tensor, eps: float,
               qkv: "torch.nn.Linear") -> Tuple[Tensor, Tensor, Tuple[int, int]]:
    """(x', qkv, qkv amax slot): x' = x + LN_cpe(t), qkv = LN_norm1(x') W^T + b in one launch -- the Block front half
    after the SubM conv (calflops.py:45-55); norm1's output stays on chip (sfx_cpe_ln_qkv_pairs)."""
    M, C = x.shape
    x_out = torch.empty_like(x)
    out = torch.empty(M, 3 * C, device=x.device, dtype=torch.float32)
    wsp, winv = weight_split(qkv.weight)
    ys = new_amax(x.device)
    call("sfx_cpe_ln_qkv_pairs", M, C, ptr(t.centre), t.ldt, ptr(t.partials), ptr(t.pair_pos), t.num_pairs, ptr(x),
         ptr(g_cpe), ptr(b_cpe), ptr(g1), ptr(b1), float(eps), ptr(x_out), wsp, winv, ptr(qkv.bias), ptr(out),
         ys[0], ys[1], stream())
    return x_out, out, ys


def window_table(offsets: Sequence[int], K: int) -> List[Tuple[int, int]]:
    """Pointcept get_padding_and_inverse as (key_start, query_start) windows over serialized positions."""
    tab = []
    start = 0
    for end in offsets:
        n = end - start
        nw = (n + K - 1) // K
        for w in range(nw):
            ks = start + w * K
            qs = ks
            if ks + K > end:  # ragged last window: padded with the preceding real points
                ks = end - K
            tab.append((ks, qs))
        start = end
    return tab


def window_table_np(offsets: Sequence[int], K: int) -> np.ndarray:
    """window_table as an int32 [num_windows, 2] array (vectorised)."""
    parts = []
    start = 0
    for end in offsets:
        n = end - start
        nw = (n + K - 1) // K
        qs = start + K * np.arange(nw, dtype=np.int64)
        ks = np.minimum(qs, end - K)  # ragged last window: padded with the preceding real points
        parts.append(np.stack([ks, qs], 1))
        start = end
    tab = np.concatenate(parts) if parts else np.zeros((0, 2), np.int64)
    return np.ascontiguousarray(tab, dtype=np.int32)


def window_table_varlen_np(offsets: Sequence[int], K: int) -> np.ndarray:
    """The flash branch's windows (Pointcept get_padding_and_inverse + cu_seqlens, patch K) as an int32
    [num_windows, 3] array of (key_start, query_start, key_count): a batch of n <= K points is one window of n keys
    (no padding), a longer one has K-key windows with the ragged last one padded by its preceding points."""
    parts = []
    start = 0
    for end in offsets:
        n = end - start
        if 0 < n <= K:
            parts.append(np.array([[start, start, n]], np.int64))
        elif n > K:
            qs = start + K * np.arange((n + K - 1) // K, dtype=np.int64)
            ks = np.minimum(qs, end - K)
            parts.append(np.stack([ks, qs, np.full_like(qs, K)], 1))
        start = end
    tab = np.concatenate(parts) if parts else np.zeros((0, 3), np.int64)
    return np.ascontiguousarray(tab, dtype=np.int32)


def window_attention_varlen(qkv: Tensor, order: Tensor, win3: Tensor, num_windows: int, K: int, heads: int,
                            channels: int, out: Optional[Tensor] = None,
                            qkv_amax: Optional[Tuple[int, int]] = None) -> Tensor:
    """Flash-mode attention (enable_flash=True, K = 1024): per-window key counts, online softmax (attention.hip);
    fp16x2 MFMA terms with an amax slot bounding |qkv|, bf16x3 otherwise (both fp32-accurate)."""
    n = qkv.shape[0]
    d = channels // heads
    if qkv.shape != (n, 3 * channels) or order.shape[0] != n or tuple(win3.shape) != (num_windows, 3):
        raise ValueError(f"window_attention_varlen: shapes qkv {tuple(qkv.shape)} order {tuple(order.shape)} "
                         f"win3 {tuple(win3.shape)} for C={channels}, {num_windows} windows")
    if out is None:
        out = torch.empty(n, channels, device=qkv.device, dtype=torch.float32)
    call("sfx_window_attention_varlen", num_windows, K, heads, d, channels, ptr(qkv), ptr(order, torch.int32),
         ptr(win3, torch.int32), float(d ** -0.5), ptr(out), *_slot_args(qkv_amax), stream())
    return out


def window_attention(qkv: Tensor, order: Tensor, win: Tensor, num_windows: int, K: int, heads: int, channels: int,
                     out: Optional[Tensor] = None, qkv_amax: Optional[Tuple[int, int]] = None) -> Tensor:
    """Windowed softmax attention (attention.hip); with an amax slot bounding |qkv| the MFMA terms are fp16x2,
    otherwise bf16x3 (both fp32-accurate)."""
    n = qkv.shape[0]
    d = channels // heads
    if out is None:
        out = torch.empty(n, channels, device=qkv.device, dtype=torch.float32)
    call("sfx_window_attention", num_windows, K, heads, d, channels, ptr(qkv), ptr(order, torch.int32),
         ptr(win, torch.int32), float(d ** -0.5), ptr(out), *_slot_args(qkv_amax), stream())
    return out


# Fused attention + output projection + residual (csrc/attn_proj.hip, ABI v15) on the eval path.  Default on the
# (channels, head_dim) where it measured faster than the attention launch + projection GEMM (config B, round 6:
# C = 64: 51 vs 58 us, C = 96: 79 vs 89 us per Block); at C = 128 / 256 one workgroup per window keeps too few
# head gathers in flight (92 vs ~80 us, 145 vs ~99 us: DESIGN.md §14).  SFX_ATTN_PROJ=0: never; =all: every
# supported shape.
_ATTN_PROJ_MODE = os.environ.get("SFX_ATTN_PROJ", "1")
_ATTN_PROJ_SHAPES = {(64, 32), (96, 24), (128, 16), (256, 16)}
_ATTN_PROJ_DEFAULT = {(64, 32), (96, 24)}


def window_attention_proj_ok(channels: int, heads: int) -> bool:
    if _ATTN_PROJ_MODE == "0":
        return False
    shapes = _ATTN_PROJ_SHAPES if _ATTN_PROJ_MODE == "all" else _ATTN_PROJ_DEFAULT
    return (channels, channels // heads) in shapes and get_precision() == "fp32"


def window_attention_proj(qkv: Tensor, order: Tensor, win: Tensor, num_windows: int, K: int, heads: int,
                          channels: int, proj: "torch.nn.Linear", x1: Tensor, qkv_amax: Tuple[int, int],
                          out: Optional[Tensor] = None) -> Tensor:
    """x1 + proj(window_attention(qkv)) in one launch (the per-head outputs stay on chip, csrc/attn_proj.hip):
    SerializedAttention's attention + proj and the Block's residual add (calflops.py:51-69).  fp16x2 MFMA terms
    (q / k / v / O scaled from the qkv amax slot, the projection weight from its cached pre-split)."""
    n = qkv.shape[0]
    d = channels // heads
    if qkv.shape != (n, 3 * channels) or order.shape[0] != n or x1.shape != (n, channels):
        raise ValueError(f"window_attention_proj: shapes qkv {tuple(qkv.shape)} order {tuple(order.shape)} "
                         f"x1 {tuple(x1.shape)} for C={channels}")
    wsp, winv = weight_split(proj.weight)
    if wsp is None:
        raise RuntimeError("window_attention_proj: the projection weight has no fp16x2 pre-split")
    if out is None:
        out = torch.empty(n, channels, device=qkv.device, dtype=torch.float32)
    px, ldx = _rows(x1)
    po, ldo = _rows(out)
    call("sfx_window_attention_proj", num_windows, K, heads, d, channels, ptr(qkv), ptr(order, torch.int32),
         ptr(win, torch.int32), float(d ** -0.5), *qkv_amax, wsp, winv, ptr(proj.bias), px, ldx, po, ldo, stream())
    return out


def _sort(keys: Tensor, vals: Optional[Tensor], begin: int, end: int) -> Tuple[Tensor, Tensor]:
    n = keys.shape[0]
    ko = torch.empty_like(keys)
    vo = torch.empty(n, device=keys.device, dtype=torch.int32)
    ws = _lib.workspace(_lib.fn("sfx_sort_workspace_bytes")(n), keys.device)
    call("sfx_sort_pairs_u64", n, ptr(keys), ptr(vals), ptr(ko), ptr(vo), begin, end, ptr(ws), ws.numel(), stream())
    return ko, vo


def _finalize(keys: Tensor, n: int, R: int, code_bits: int) -> Tuple[Tensor, Tensor]:
    _, pos = _sort(keys, None, 0, code_bits + 2)
    order = torch.empty(R, n, device=keys.device, dtype=torch.int32)
    inverse = torch.empty(R, n, device=keys.device, dtype=torch.int32)
    call("sfx_serialize_finalize", n, R, ptr(pos), ptr(order), ptr(inverse), stream())
    return order, inverse


def serialize(grid_coord: Tensor, batch: Optional[Tensor], depth: int, code_bits: int,
              orders: Sequence[str]) -> Tuple[Tensor, Tensor, Tensor]:
    """Codes [R,n] int64 + stable argsort order / inverse [R,n] int32 for every order type (one radix sort)."""
    n = grid_coord.shape[0]
    R = len(orders)
    t = [ORDER_TYPES[o] for o in orders] + [0] * (4 - R)
    codes = torch.empty(R, n, device=grid_coord.device, dtype=torch.int64)
    keys = torch.empty(R * n, device=grid_coord.device, dtype=torch.int64)
    call("sfx_serialize_keys", n, ptr(grid_coord, torch.int32), ptr(batch), depth, R, t[0], t[1], t[2], t[3],
         code_bits, ptr(codes), ptr(keys), stream())
    order, inverse = _finalize(keys, n, R, code_bits)
    return codes, order, inverse


def serialize_permute(codes: Tensor, order: Tensor, inverse: Tensor, grid: Tensor, coord: Tensor):
    """Renumber the points by serialized order row 0 (sfx_serialize_permute): -> (codes, order, inverse, grid,
    coord) in the new numbering; new point i is old point order[0][i]."""
    R, n = codes.shape
    cp, op, ip = torch.empty_like(codes), torch.empty_like(order), torch.empty_like(inverse)
    gp = torch.empty_like(grid)
    xp = torch.empty(n, 3, device=coord.device, dtype=torch.float32)
    call("sfx_serialize_permute", n, R, ptr(order, torch.int32), ptr(inverse, torch.int32), ptr(codes, torch.int64),
         ptr(grid, torch.int32), ptr(coord, torch.float32), ptr(cp), ptr(op), ptr(ip), ptr(gp), ptr(xp), stream())
    return cp, op, ip, gp, xp


def scan_i32(x: Tensor, inclusive: bool = True, total: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
    n = x.shape[0]
    out = torch.empty_like(x)
    if total is None:
        total = torch.empty(1, device=x.device, dtype=torch.int32)
    ws = _lib.workspace(_lib.fn("sfx_scan_workspace_bytes")(n), x.device)
    call("sfx_scan_i32", n, ptr(x), ptr(out), 1 if inclusive else 0, ptr(ws), ws.numel(), ptr(total), stream())
    return out, total


def pool_geometry_begin(codes: Tensor, order: Tensor, pooling_depth: int):
    """First half of pool_geometry: run flags + their scan, and an asynchronous read of the per-row run counts
    (work the caller enqueues before pool_geometry_end overlaps the host wait)."""
    R, n = codes.shape
    flags = torch.empty(R * n, device=codes.device, dtype=torch.int32)
    call("sfx_pool_run_flags", n, R, ptr(order, torch.int32), ptr(codes, torch.int64), 3 * pooling_depth,
         ptr(flags), stream())
    pos, _ = scan_i32(flags)
    return flags, pos, _lib.HostRead(pos.view(R, n)[:, -1])


def pool_counts_begin(codes: Tensor, order: Tensor, shifts: Sequence[int]) -> "_lib.HostRead":
    """The cluster counts of every pooling of a forward, from the stage-0 serialization alone: codes are
    hierarchical (a pooling keeps the head's code >> 3pd), so the m of the pooling reached after cumulative shift
    k is the number of runs of code0 >> k along serialized row 0 -- one flag pass + scan per pooling, read back in
    one asynchronous copy.  The forward then never waits for a pooled count (pool_geometry_end(m=...))."""
    n = codes.shape[1]
    counts = torch.empty(max(len(shifts), 1), device=codes.device, dtype=torch.int32)
    for k in range(0, len(shifts), 8):  # one launch for up to 8 poolings (sfx_pool_run_counts)
        sh = list(shifts[k:k + 8])
        call("sfx_pool_run_counts", n, ptr(order[0], torch.int32), ptr(codes[0], torch.int64),
             ctypes.cast((ctypes.c_int * len(sh))(*sh), ctypes.c_void_p), len(sh), counts[k:].data_ptr(), stream())
    return _lib.HostRead(counts)


def check_pool_runs(ends: Sequence[int], m: int) -> None:
    runs = [ends[0]] + [ends[r] - ends[r - 1] for r in range(1, len(ends))]
    if any(c != m for c in runs):
        raise RuntimeError(f"sfx pooling: order rows count cluster runs {runs}, expected {m}; the serialization codes "
                           "are not hierarchical (code >> 3 must be the parent cell's code)")


def pool_geometry_end(state, codes: Tensor, order: Tensor, row0: int, pooling_depth: int, grid_coord: Tensor,
                      batch: Optional[Tensor], code_bits: int, m: Optional[int] = None,
                      deferred: Optional[list] = None):
    """m (from pool_counts_begin) skips the wait for this pooling's count; the per-row run counts are then checked
    later by the caller from `deferred` ((HostRead, m) pairs)."""
    flags, pos, ends_rd = state
    R, n = codes.shape
    dev = codes.device
    shift = 3 * pooling_depth
    if m is None:
        ends = ends_rd.get()  # the pooled point count sizes every later buffer
        m = ends[0]
        check_pool_runs(ends, m)
    else:
        deferred.append((ends_rd, m))
    cluster = torch.empty(n, device=dev, dtype=torch.int32)
    sidx = torch.empty(n, device=dev, dtype=torch.int32)
    idx_ptr = torch.empty(m + 1, device=dev, dtype=torch.int32)
    head = torch.empty(m, device=dev, dtype=torch.int32)
    call("sfx_pool_assign_runs", n, m, row0, ptr(order), ptr(pos), ptr(flags), ptr(cluster), ptr(idx_ptr),
         ptr(head), ptr(sidx), stream())
    new_order = torch.empty(R, m, device=dev, dtype=torch.int32)
    new_inverse = torch.empty(R, m, device=dev, dtype=torch.int32)
    call("sfx_pool_reorder", n, m, R, ptr(order), ptr(pos), ptr(flags), ptr(cluster), ptr(new_order),
         ptr(new_inverse), stream())
    new_codes = torch.empty(R, m, device=dev, dtype=torch.int64)
    new_grid = torch.empty(m, 3, device=dev, dtype=torch.int32)
    new_batch = torch.empty(m, device=dev, dtype=torch.int32) if batch is not None else None
    call("sfx_pool_gather", m, n, R, ptr(head), ptr(codes), pooling_depth, ptr(grid_coord), ptr(batch),
         code_bits - shift, ptr(new_codes), None, ptr(new_grid), ptr(new_batch), stream())
    return sidx, cluster, idx_ptr, m, new_codes, new_order, new_inverse, new_grid, new_batch


def pool_geometry(codes: Tensor, order: Tensor, row0: int, pooling_depth: int, grid_coord: Tensor,
                  batch: Optional[Tensor], code_bits: int):
    """SerializedPooling's integer half without a sort (serialize.hip): runs of equal code >> 3pd along the
    parent's serialized orders are the clusters, in ascending pooled-code order for every row.
    -> (sorted_idx, cluster, idx_ptr, m, new codes [R,m], new order, new inverse, new grid, new batch)."""
    st = pool_geometry_begin(codes, order, pooling_depth)
    return pool_geometry_end(st, codes, order, row0, pooling_depth, grid_coord, batch, code_bits)


def segment_max_affine_act(x: Tensor, idx_ptr: Tensor, sorted_idx: Tensor, m: int, scale: Optional[Tensor],
                           shift: Optional[Tensor], act: int) -> Tensor:
    C = x.shape[1]
    out = torch.empty(m, C, device=x.device, dtype=torch.float32)
    call("sfx_segment_max_affine_act", m, C, ptr(idx_ptr), ptr(sorted_idx), ptr(x), ptr(scale), ptr(shift), act,
         ptr(out), stream())
    return out


def segment_mean(x: Tensor, idx_ptr: Tensor, sorted_idx: Tensor, m: int) -> Tensor:
    D = x.shape[1]
    out = torch.empty(m, D, device=x.device, dtype=torch.float32)
    call("sfx_segment_mean", m, D, ptr(idx_ptr), ptr(sorted_idx), ptr(x.contiguous()), ptr(out), stream())
    return out


PAIR_LISTS = os.environ.get("SFX_PAIR_LISTS", "1") != "0"  # 0: the older flag / scan / fill pair builder
LN_COMPACT = os.environ.get("SFX_LN_COMPACT", "1") != "0"  # 0: the pair-sum LayerNorm reads pair_pos [n][27]


class PairLists:
    """Offset-major SubM pair lists of one map (sfx_subm_pairs): pair_in / pair_out, the 28 per-offset prefixes (read
    back asynchronously; the first conv that needs them waits for that copy only) and the inverted index pair_pos.
    centre=True also lists the centre offset k = 13 (the eval conv's single pair launch, ABI v15)."""

    def __init__(self, nbr: Tensor, centre: bool):
        n = nbr.shape[0]
        dev = nbr.device
        cap = max(1, (27 if centre else 26) * n)
        self.centre = centre
        self.pair_in = torch.empty(cap, device=dev, dtype=torch.int32)
        self.pair_out = torch.empty(cap, device=dev, dtype=torch.int32)
        self.off_dev = torch.empty(28, device=dev, dtype=torch.int32)
        if PAIR_LISTS:
            # lists and the inverted index pair_pos in one call (ABI v16: per-workgroup counts, no host value needed)
            # with the compacted positions the pair-sum LayerNorm reads (present pairs first, count in column 31);
            # then the [n][27] index is only built if asked for (pair_pos, e.g. SubmPartials.total())
            self.cpos = torch.empty(max(1, n), 32, device=dev, dtype=torch.int32) if LN_COMPACT else None
            self._pos = None if LN_COMPACT else torch.empty(max(1, n), 27, device=dev, dtype=torch.int32)
            ws = _lib.workspace(_lib.fn("sfx_subm_pair_lists_workspace_bytes")(n), dev)
            call("sfx_subm_pair_lists", n, ptr(nbr), ptr(ws), ws.numel(), ptr(self.pair_in), ptr(self.pair_out),
                 ptr(self.off_dev), ptr(self._pos), ptr(self.cpos), 1 if centre else 0, stream())
        else:  # the v6 / v15 pair (flags over [27][n] + scan + fill; pair_pos on first use, after the offsets read)
            self._pos = None
            self.cpos = None
            ws = _lib.workspace(_lib.fn("sfx_subm_pairs_workspace_bytes")(n), dev)
            call("sfx_subm_pairs", n, ptr(nbr), ptr(ws), ws.numel(), ptr(self.pair_in), ptr(self.pair_out),
                 ptr(self.off_dev), 1 if centre else 0, stream())
        self._rd = _lib.HostRead(self.off_dev)
        self._n = n
        self._off = None
        self._off_c = None

    def off_ready(self) -> bool:
        return self._off is not None

    @property
    def pair_off(self) -> List[int]:
        if self._off is None:
            self._off = self._rd.get()
        return self._off

    @property
    def off_host(self):
        if self._off_c is None:
            self._off_c = (ctypes.c_int * 28)(*self.pair_off)
        return self._off_c

    @property
    def num_pairs(self) -> int:
        return self.pair_off[27]

    @property
    def pair_pos(self) -> Tensor:
        """[n, 27] inverted pair index (written with the lists by sfx_subm_pair_lists; SFX_PAIR_LISTS=0: built on
        first use by sfx_subm_pair_pos)."""
        if self._pos is None:
            pos = torch.empty(self._n, 27, device=self.pair_in.device, dtype=torch.int32)
            call("sfx_subm_pair_pos", self._n, self.num_pairs, ptr(self.pair_out), ptr(self.off_dev), ptr(pos),
                 stream())
            self._pos = pos
        return self._pos


class SubmMap:
    """Per-stage SubMConv3d indice map (indice_key=stage{s}): nbr [n,27] + offset-major pair lists (PairLists), built
    on first use (subm_neighbors(with_pairs=True) builds the preferred kind right away): the fused conv
    (subm_cpe_ln) reads nbr only.  Two kinds of lists: without the centre offset (the atomic conv, the training
    backward) and with it (centre_pref: the eval conv's single pair launch)."""

    def __init__(self, nbr: Tensor, mask: Optional[Tensor], centre_pref: bool = False):
        self.nbr, self.mask = nbr, mask
        self.centre_pref = centre_pref
        self._lists = {}
        self._order = None

    def lists(self, centre: bool = False) -> PairLists:
        pl = self._lists.get(centre)
        if pl is None:
            pl = self._lists[centre] = PairLists(self.nbr, centre)
        return pl

    def ensure_pairs(self) -> "SubmMap":
        self.lists(False)
        return self

    @property
    def pair_in(self) -> Tensor:
        return self.lists(False).pair_in

    @property
    def pair_out(self) -> Tensor:
        return self.lists(False).pair_out

    @property
    def pair_pos(self) -> Tensor:
        return self.lists(False).pair_pos

    @property
    def order(self) -> Tensor:
        """The fused conv's row order (sfx_subm_order_keys + a 2-pass radix sort): rows grouped by neighbour mask,
        built once per map (every conv of the stage shares it)."""
        if self._order is None:
            n = self.nbr.shape[0]
            keys = torch.empty(n, device=self.nbr.device, dtype=torch.int64)
            call("sfx_subm_order_keys", n, ptr(self.nbr), ptr(keys), stream())
            _, self._order = _sort(keys, None, 0, 16)
        return self._order

    def pair_off_ready(self) -> bool:
        """Whether the (centre-free) pair offsets are already on the host (reading them costs no wait)."""
        return self.lists(False).off_ready()

    @property
    def pair_off(self) -> List[int]:
        return self.lists(False).pair_off

    @property
    def _off_host(self):
        return self.lists(False).off_host

    @property
    def shape(self):
        return self.nbr.shape

    @property
    def num_pairs(self) -> int:
        return self.lists(False).num_pairs


SUBM_MASK = os.environ.get("SFX_SUBM_MASK", "0") == "1"


def subm_neighbors(grid_coord: Tensor, batch: Optional[Tensor], with_pairs: bool = True, centre: bool = False):
    """27-neighbour map; with_pairs also builds the offset-major pair lists (their offsets read back asynchronously):
    with the centre offset when `centre` (the eval forward's maps), else without."""
    n = grid_coord.shape[0]
    dev = grid_coord.device
    l2 = _lib.fn("sfx_subm_table_log2")(n)
    tk = torch.empty(1 << l2, device=dev, dtype=torch.int64)
    tv = torch.empty(1 << l2, device=dev, dtype=torch.int32)
    nbr = torch.empty(n, 27, device=dev, dtype=torch.int32)
    # no neighbour bitmask by default: nothing reads it (the fused conv's row order comes from nbr,
    # sfx_subm_order_keys), and the query would pay one atomicOr per present neighbour for it (SFX_SUBM_MASK=1: built)
    mask = torch.empty(n, device=dev, dtype=torch.int32) if SUBM_MASK else None
    call("sfx_subm_neighbors", n, ptr(grid_coord, torch.int32), ptr(batch), l2, ptr(tk), ptr(tv), ptr(nbr), ptr(mask),
         None, stream())
    smap = SubmMap(nbr, mask, centre_pref=centre)
    if with_pairs:
        smap.lists(centre)
    return smap


# eval-path SubM convs: store per-pair partials and sum them in the consumer (default), or add them atomically
SUBM_PARTIALS = os.environ.get("SFX_SUBM_ATOMIC", "0") != "1"
# the eval forward's maps list the centre offset with the pairs: each conv is ONE pair launch, the centre's products
# being partial rows like the other offsets' (was a separate centre GEMM launch); SFX_SUBM_CENTRE_PAIRS=0 restores it
SUBM_CENTRE_PAIRS = os.environ.get("SFX_SUBM_CENTRE_PAIRS", "1") != "0"
# the first conv of a new SubM map enqueues its centre GEMM before waiting for the pair offsets
SUBM_CENTRE_FIRST = os.environ.get("SFX_SUBM_CENTRE_FIRST", "1") != "0"
PAIRS_LN_CHANNELS = (64, 96, 128, 256, 512)  # the channel counts sfx_cpe_residual_ln_pairs has kernels for


def subm_partials_ok(x: Tensor, smap: "SubmMap", cout: int) -> bool:
    """Whether the atomic-free SubM form can run for this launch: its consumer (sfx_cpe_residual_ln_pairs) needs
    C in PAIRS_LN_CHANNELS, 16-byte aligned contiguous rows and partials below the 2 GiB buffer range; other
    launches (e.g. enc_dim=32's C=32 stage 0, reference pointtransformer_v3.py:113) take the atomic form."""
    # the 2 GiB partials bound from 27 n (no host wait for the pair count) unless that bound is too coarse
    return (SUBM_PARTIALS and cout in PAIRS_LN_CHANNELS and x.shape[1] == cout and x.is_contiguous()
            and x.data_ptr() % 16 == 0 and (27 * smap.nbr.shape[0] * cout * 4 + 64 < 0x7ffffff0
                                            or smap.lists(smap.centre_pref).num_pairs * cout * 4 + 64 < 0x7ffffff0))


# Block.cpe + shortcut + norm1 of the eval forward in one launch, the conv summed in MFMA registers over all 27
# offsets (csrc/subm_fused.hip).  Default ("auto"): on maps of at least SUBM_FUSED_MIN_ROWS points at C <= 128, where
# it beats the offset-major pair GEMM + pair-sum LayerNorm (config-E stages 0-2: 12-28 % faster per conv; the smaller
# maps of config B and every C = 256 map measured slower -- profiles/r05_subm_fused_sizes.txt).
# SFX_SUBM_FUSED=1: on every map whose C is in SFX_SUBM_FUSED_CHANNELS; SFX_SUBM_FUSED=0: never.
SUBM_FUSED_MODE = os.environ.get("SFX_SUBM_FUSED", "auto")
SUBM_FUSED_MIN_ROWS = int(os.environ.get("SFX_SUBM_FUSED_MIN_ROWS", "120000"))
SUBM_FUSED_AUTO_MAX_C = 128
SUBM_FUSED_KERNELS = (64, 96, 128, 256)  # the channel counts sfx_subm_cpe_ln has kernels for
SUBM_FUSED_CHANNELS = tuple(int(c) for c in os.environ.get("SFX_SUBM_FUSED_CHANNELS", "64,96,128,256").split(",")
                            if c and int(c) in SUBM_FUSED_KERNELS)


def subm_fused_ok(C: int, n: Optional[int] = None) -> bool:
    """Whether an eval Block on a map of n points with C channels runs sfx_subm_cpe_ln (n None: unknown size,
    the auto rule then says no)."""
    if SUBM_FUSED_MODE == "0" or C not in SUBM_FUSED_CHANNELS:
        return False
    if SUBM_FUSED_MODE == "1":
        return True
    return n is not None and n >= SUBM_FUSED_MIN_ROWS and C <= SUBM_FUSED_AUTO_MAX_C


def subm_cpe_pack(wf: Tensor) -> Tuple[Tensor, Tensor]:
    """Folded CPE conv weight W' [C, 27*C] -> (fp16x2 fragment stream, inverse column scales) for subm_cpe_ln."""
    C = wf.shape[0]
    nb = int(_lib.fn("sfx_subm_cpe_pack_bytes")(C))
    if nb == 0 or wf.shape[1] != 27 * C:
        raise RuntimeError(f"subm_cpe_pack: no fused conv for C={C}")
    wpk = torch.empty(nb // 4, device=wf.device, dtype=torch.float32)
    winv = torch.empty(C, device=wf.device, dtype=torch.float32)
    ws = torch.empty(C, device=wf.device, dtype=torch.float32)
    call("sfx_subm_cpe_pack", C, ptr(wf.contiguous()), ptr(wpk), ptr(winv), ptr(ws), stream())
    return wpk, winv


def subm_rowexp(x: Tensor) -> Tensor:
    """Per-row fp16x2 exponents of a conv input (sfx_subm_rowexp): x_j * 2^e_j has its maximum in [2^14, 2^15)."""
    n, C = x.shape
    e = torch.empty(n, device=x.device, dtype=torch.int32)
    call("sfx_subm_rowexp", n, C, ptr(x), ptr(e), stream())
    return e


def subm_cpe_ln(xc: Tensor, x: Tensor, smap: "SubmMap", wpk: Tensor, winv: Tensor, bias: Tensor, g_cpe: Tensor,
                b_cpe: Tensor, g1: Tensor, b1: Tensor, eps: float,
                rowexp: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
    """x1 = x + LN_cpe(SubMConv'(xc)), h = LN1(x1) in one launch (csrc/subm_fused.hip; C in SUBM_FUSED_KERNELS)."""
    n, C = x.shape
    if xc.shape != x.shape or not (xc.is_contiguous() and x.is_contiguous()):
        raise RuntimeError("subm_cpe_ln: contiguous [n, C] inputs expected")
    x1 = torch.empty_like(x)
    h = torch.empty_like(x)
    call("sfx_subm_cpe_ln", n, C, ptr(xc), ptr(x), ptr(smap.nbr), ptr(smap.order),
         ptr(subm_rowexp(xc) if rowexp is None else rowexp), ptr(wpk),
         ptr(winv), ptr(bias), ptr(g_cpe), ptr(b_cpe), ptr(g1), ptr(b1), float(eps), ptr(x1), ptr(h), stream())
    return x1, h


_ZERO_OFFS = (ctypes.c_int * 28)()  # pair offsets of a centre-only sfx_subm_conv_partials call


class SubmPartials:
    """Atomic-free SubM conv output: centre [n, Cout] (bias + centre offset) and partials [num_pairs, Cout] (one row
    per (offset, output) pair), summed per output row by the consumer (cpe_residual_ln) or by `total()`.  ldt = 0:
    `centre` is the bias [Cout] alone and the centre offset's products are partial rows (pair lists with the centre)."""

    def __init__(self, centre: Tensor, partials: Tensor, pair_pos, num_pairs: int, ldt: Optional[int] = None,
                 cpos: Optional[Tensor] = None):
        """pair_pos: the [n][27] index, or the PairLists that builds it on first use."""
        self.centre, self.partials, self._pair_pos, self.num_pairs = centre, partials, pair_pos, num_pairs
        self.ldt = centre.shape[-1] if ldt is None else ldt
        self.cpos = cpos  # compacted positions (PairLists.cpos) or None

    @property
    def pair_pos(self) -> Tensor:
        return self._pair_pos.pair_pos if isinstance(self._pair_pos, PairLists) else self._pair_pos

    def total(self) -> Tensor:
        """The conv output, summed in the consumer's order (ascending offsets after the centre / the bias)."""
        n = self.pair_pos.shape[0]
        out = self.centre.expand(n, -1).clone() if self.ldt == 0 else self.centre.clone()
        pos = self.pair_pos.long()
        for k in range(27):
            sel = pos[:, k] >= 0
            if bool(sel.any()):
                out[sel] += self.partials[pos[sel, k]]
        return out


def subm_conv(x: Tensor, smap: "SubmMap", weight: Tensor, bias: Optional[Tensor],
              out: Optional[Tensor] = None, x_amax: Optional[Tuple[int, int]] = None,
              w_amax: Optional[Tuple[int, int]] = None, partials: bool = False):
    """SubMConv3d(k=3): dense centre GEMM + offset-major pair GEMM with atomic accumulation (x_amax / w_amax:
    amax slots bounding |x| and the whole weight; None: measured by the library).  partials=True: the pair
    products are stored per pair instead (no atomics) and a SubmPartials is returned for cpe_residual_ln."""
    n, cin = x.shape
    cout = weight.shape[0]
    if out is None:
        out = torch.empty(n, cout, device=x.device, dtype=torch.float32)
    px, ldx = _rows(x)
    po, ldo = _rows(out)
    if partials:
        wsp = weight_split(weight)
        if smap.centre_pref and SUBM_CENTRE_PAIRS:  # one pair launch over all 27 offsets (the lists carry the centre)
            pl = smap.lists(True)
            npairs = pl.num_pairs
            part = torch.empty(max(1, npairs), cout, device=x.device, dtype=torch.float32)
            call("sfx_subm_conv_partials_pairs", n, cin, cout, px, ldx, ptr(smap.nbr), ptr(weight), ptr(bias),
                 ptr(pl.pair_in), ptr(pl.pair_out), pl.off_host, po, ldo, ptr(part), cout, *wsp, stream())
            b = bias if bias is not None else torch.zeros(cout, device=x.device, dtype=torch.float32)
            return SubmPartials(b.contiguous(), part, pl, npairs, ldt=0, cpos=pl.cpos)
        if SUBM_CENTRE_FIRST and not smap.pair_off_ready():  # centre GEMM first, then wait for the pair offsets
            call("sfx_subm_conv_partials", n, cin, cout, px, ldx, ptr(smap.nbr), ptr(weight), ptr(bias), None, None,
                 _ZERO_OFFS, po, ldo, None, cout, *wsp, stream())
            npairs = smap.num_pairs
            part = torch.empty(max(1, npairs), cout, device=x.device, dtype=torch.float32)
            call("sfx_subm_conv_partials_pairs", n, cin, cout, px, ldx, ptr(smap.nbr), ptr(weight), ptr(bias),
                 ptr(smap.pair_in), ptr(smap.pair_out), smap._off_host, po, ldo, ptr(part), cout, *wsp, stream())
            return SubmPartials(out, part, smap.lists(False), npairs, cpos=smap.lists(False).cpos)
        npairs = smap.num_pairs
        part = torch.empty(max(1, npairs), cout, device=x.device, dtype=torch.float32)
        call("sfx_subm_conv_partials", n, cin, cout, px, ldx, ptr(smap.nbr), ptr(weight), ptr(bias),
             ptr(smap.pair_in), ptr(smap.pair_out), smap._off_host, po, ldo, ptr(part), cout, *wsp, stream())
        return SubmPartials(out, part, smap.lists(False), npairs, cpos=smap.lists(False).cpos)
    call("sfx_subm_conv", n, cin, cout, px, ldx, ptr(smap.nbr), ptr(weight), ptr(bias), ptr(smap.pair_in),
         ptr(smap.pair_out), smap._off_host, po, ldo, *_slot_args(x_amax), *_slot_args(w_amax),
         *weight_split(weight), stream())
    return out


def move_rows(src: Tensor, idx: Tensor, dst: Optional[Tensor] = None, scatter: bool = False) -> Tensor:
    """dst[i] = src[idx[i]] (gather) or dst[idx[i]] = src[i] (scatter) for the rows of a 2-D (or 1-D) tensor of
    4- or 8-byte elements (sfx_move_rows)."""
    s2 = src if src.dim() == 2 else src.reshape(src.shape[0], -1)
    esz = s2.element_size()
    if esz not in (4, 8) or s2.stride(1) != 1:
        raise RuntimeError("move_rows: rows of 4- or 8-byte elements, unit column stride")
    n = idx.shape[0]
    if dst is None:
        if scatter:
            raise RuntimeError("move_rows: scatter needs a destination")
        dst = torch.empty((n,) + tuple(src.shape[1:]), device=src.device, dtype=src.dtype)
    d2 = dst if dst.dim() == 2 else dst.reshape(dst.shape[0], -1)
    words = s2.shape[1] * esz // 4
    call("sfx_move_rows", n, words, s2.data_ptr(), s2.stride(0) * esz // 4, ptr(idx, torch.int32), d2.data_ptr(),
         d2.stride(0) * esz // 4, 1 if scatter else 0, stream())
    return dst


def gs_pack(gs: dict, feat_out: Tensor, grid_resolution: float, grid_out: Optional[Tensor],
            grid_max: Optional[Tensor] = None) -> None:
    """FeaturePredictor batchify (feature_predictor.py:137-156) into a strided feature view."""
    n = gs["means"].shape[0]

    def rp(t):
        t2 = t if t.dim() == 2 else t.reshape(t.shape[0], -1)
        if t2.stride(-1) != 1:
            t2 = t2.contiguous()
        return t2.data_ptr(), t2.stride(0), t2

    keep = []
    args = []
    for k in ["means", "scales", "opacities", "quats", "features_dc"]:
        p_, l_, t_ = rp(gs[k])
        keep.append(t_)
        args += [p_, l_]
    rest = gs.get("features_rest")
    if rest is not None:
        p_, l_, t_ = rp(rest if rest.is_contiguous() else rest.contiguous())
        keep.append(t_)
        rd = t_.shape[1]
    else:
        p_, l_, rd = None, 0, 0
    pf, ldf = _rows(feat_out)
    call("sfx_gs_pack", n, *args, p_, l_, rd, float(grid_resolution), pf, ldf, ptr(grid_out), ptr(grid_max),
         stream())
