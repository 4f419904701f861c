"""Python side of the gemm2 experiment (experiments/gemm2/gemm2.hip): operand planes and the LDS-DMA GEMM.
Built into its own library, not libsfx.so (measured slower than csrc/gemm.hip inside the refine:
profiles/r03_gemm2_block_ab.txt; DESIGN.md "gemm2").  Build: bash experiments/gemm2/build.sh; the functions below
expect `SFX_LIB=experiments/gemm2/libsfx_gemm2.so` (libsfx plus gemm2 and the planes LayerNorm of norm_planes.patch).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
from torch import Tensor

from splatformer_amd import _lib
from splatformer_amd._lib import I, L, P, F, call, ptr, stream
from splatformer_amd.ptv3_ops import ACT_NONE, _rows, _slot_args, new_amax

_lib.register("sfx_split_planes", [I, I, I, P, L, P, L, P, P])
_lib.register("sfx_gemm2", [I, I, I, I, P, L, P, I, P, I, P, L, P, P, P, P, I, I, P, L, P, P, L, P, I, P])
_lib.register("sfx_gemm2_pairs", [I, I, P, L, P, I, P, P, P, L, P, P, L, P])
_lib.register("sfx_gemm2_ok", [I, I, P, P, P, P, P, L, P, L])

class Planes:
    """fp16x2 planes of a fp32 matrix [rows, K]: buf = [2][rows][Kp] fp16 (h then l terms of X * 2^e_r, K padded
    to Kp = ceil32(K) with zeros), inv[r] = 2^-e_r (sfx_split_planes)."""
    __slots__ = ("buf", "inv", "rows", "K", "Kp")

    def __init__(self, buf: Tensor, inv: Tensor, rows: int, K: int, Kp: int):
        self.buf, self.inv, self.rows, self.K, self.Kp = buf, inv, rows, K, Kp

    @property
    def plane(self) -> int:
        return self.rows * self.Kp


def split_planes(x: Tensor, rows: Optional[int] = None) -> Planes:
    rows = x.shape[0] if rows is None else rows
    K = x.shape[1]
    Kp = (K + 31) // 32 * 32
    pa, lda = _rows(x)
    buf = torch.empty(2 * max(rows, 1) * Kp, device=x.device, dtype=torch.float16)
    inv = torch.empty(max(rows, 1), device=x.device, dtype=torch.float32)
    call("sfx_split_planes", rows, K, Kp, pa, lda, ptr(buf), max(rows, 1) * Kp, ptr(inv), stream())
    return Planes(buf, inv, max(rows, 1), K, Kp)


def new_planes(rows: int, K: int, device) -> Planes:
    Kp = (K + 31) // 32 * 32
    r = max(rows, 1)
    return Planes(torch.empty(2 * r * Kp, device=device, dtype=torch.float16),
                  torch.empty(r, device=device, dtype=torch.float32), r, K, Kp)


def weight_planes(w: Tensor) -> Planes:
    """Planes of a weight [N, K], cached on the tensor until its storage or version changes."""
    key = (w.data_ptr(), w._version, tuple(w.shape))
    c = w.__dict__.get("_sfx_wplanes")
    if c is not None and c[0] == key:
        return c[1]
    p = split_planes(w.reshape(w.shape[0], -1))
    w.__dict__["_sfx_wplanes"] = (key, p)
    return p


def linear2(x, weight: Tensor, bias: Optional[Tensor] = None, *, act: int = ACT_NONE, act_ncols: int = -1,
            scale: Optional[Tensor] = None, shift: Optional[Tensor] = None, residual: Optional[Tensor] = None,
            residual_idx: Optional[Tensor] = None, out: Optional[Tensor] = None,
            gather_idx: Optional[Tensor] = None, rows: Optional[int] = None, y_amax: bool = False):
    """`linear` on pre-split planes (sfx_gemm2): x is a Tensor (split here) or Planes; gather_idx [M] / [M, 1]
    selects A rows (-1 = zero row)."""
    wp = weight_planes(weight)
    xp = x if isinstance(x, Planes) else split_planes(x)
    if xp.Kp != wp.Kp:
        raise RuntimeError(f"linear2: x has {xp.K} features, weight expects {wp.K}")
    N = weight.shape[0]
    M = (gather_idx.shape[0] if gather_idx is not None else (xp.rows if rows is None else rows))
    if out is None:
        out = torch.empty(M, N, device=weight.device, dtype=torch.float32)
    py, ldy = _rows(out)
    pr, ldr = _rows(residual) if residual is not None else (None, 0)
    ys = new_amax(out.device) if y_amax else None
    gs = gather_idx.stride(0) if gather_idx is not None else 1
    call("sfx_gemm2", 1 if gather_idx is not None else 0, M, N, xp.Kp, ptr(xp.buf), xp.plane, ptr(xp.inv), xp.rows,
         ptr(gather_idx), gs, ptr(wp.buf), wp.plane, ptr(wp.inv), ptr(bias), ptr(scale), ptr(shift), act, act_ncols,
         pr, ldr, ptr(residual_idx), py, ldy, *_slot_args(ys), stream())
    return (out, ys) if y_amax else out




# ---- LayerNorm outputs as planes (norm_planes.patch) ----------------------------------------------------------
_lib.register("sfx_layernorm_planes", [I, I, P, L, P, P, F, P, L, P, P])
_lib.register("sfx_cpe_residual_ln_planes", [I, I, P, P, P, L, P, P, P, P, P, F, P, P, L, P, P])


def layernorm_planes(x: Tensor, gamma: Tensor, beta: Tensor, eps: float) -> Planes:
    """LayerNorm of x [M, C] written as fp16x2 Planes for linear2 (sfx_layernorm_planes)."""
    M, C = x.shape
    px, ldx = _rows(x)
    hp = new_planes(M, C, x.device)
    call("sfx_layernorm_planes", M, C, px, ldx, ptr(gamma), ptr(beta), float(eps), ptr(hp.buf), hp.plane,
         ptr(hp.inv), stream())
    return hp


def cpe_residual_ln_planes(t: Tensor, x: Tensor, g_cpe, b_cpe, g1, b1, eps: float):
    """x' = x + LN_cpe(t), h = LN_norm1(x') as Planes (t: the conv output, no pair partials)."""
    M, C = x.shape
    x_out = torch.empty_like(x)
    hp = new_planes(M, C, x.device)
    call("sfx_cpe_residual_ln_planes", M, C, ptr(t), None, None, 0, ptr(x), ptr(g_cpe), ptr(b_cpe), ptr(g1), ptr(b1),
         float(eps), ptr(x_out), ptr(hp.buf), hp.plane, ptr(hp.inv), stream())
    return x_out, hp
