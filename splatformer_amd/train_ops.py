"""Device ops of the refiner's training step (configs C/D): typed wrappers over the libsfx C-ABI.

Backward GEMMs (sfx_linear_bwd_data / sfx_linear_wgrad), the SubMConv3d input gradient, window-attention
backward, LayerNorm / train-mode BatchNorm forward+backward, pooling reductions and the Adam step.
Same rules as ptv3_ops: torch allocates, HIP computes, no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Tuple

import torch
from torch import Tensor

from . import _lib
from ._lib import F, I, L, P, Z, call, ptr, stream
from .ptv3_ops import _rows, weight_split

D = C.c_double

_lib.register("sfx_linear_bwd_data", [I, I, I, P, L, P, L, P, I, I, P, L, P, L, I, P, P, P])
_lib.register("sfx_linear_wgrad", [I, I, I, P, L, P, L, P, L, P, P])
_lib.register("sfx_transpose", [I, I, P, L, P, L, P])
_lib.register("sfx_subm_conv_bwd_data", [I, I, I, P, L, P, P, P, P, P, P, P, L, P, P, P])
_lib.register("sfx_window_attention_bwd", [I, I, I, I, I, P, P, P, F, P, P, P, P, P])
_lib.register("sfx_window_attention_varlen_bwd", [I, I, I, I, I, P, P, P, F, P, P, P, P])
_lib.register("sfx_layernorm_bwd", [I, I, P, L, P, P, L, P, L, F, P, L, P])
_lib.register("sfx_cpe_ln_bwd", [I, I, P, P, P, P, P, P, F, P, P, P])
_lib.register("sfx_colsum2_workspace_bytes", [I, I], Z)
_lib.register("sfx_bn_stats", [I, I, P, L, P, Z, P, P])
_lib.register("sfx_bn_finalize", [I, D, P, P, P, F, F, P, P, P, P, P, P, P])
_lib.register("sfx_affine_act", [I, I, P, L, P, P, I, P, L, P, P, L, P])
_lib.register("sfx_bn_act_bwd_reduce", [I, I, P, L, P, P, P, P, I, P, L, P, Z, P, P])
_lib.register("sfx_bn_act_bwd_apply", [I, I, P, L, P, P, P, P, I, P, L, P, D, P, L, I, P])
_lib.register("sfx_segment_max_arg", [I, I, P, P, P, P, P, P])
_lib.register("sfx_segment_max_bwd", [I, I, P, P, P, P])
_lib.register("sfx_segment_sum", [I, I, P, P, P, L, P, P])
_lib.register("sfx_act_bwd", [I, I, P, L, P, L, I, I, P, L, P])
_lib.register("sfx_sumsq", [L, P, P, P])
_lib.register("sfx_clip_coef", [P, F, P, P, P])
_lib.register("sfx_adam_step", [L, P, P, P, P, P, F, F, F, F, F, I, P])
_lib.register("sfx_drop_mask", [L, F, C.c_ulonglong, P, P])

DACT_NONE, DACT_GELU, DACT_RELU, DACT_TANH_OUT = 0, 1, 2, 3
_ATTN_EXACT = os.environ.get("SFX_ATTN_PREC", "")[:1] == "f"  # (read once, as attention.hip does)


def transpose(x: Tensor) -> Tensor:
    rows, cols = x.shape
    px, ldx = _rows(x)
    out = torch.empty(cols, rows, device=x.device, dtype=torch.float32)
    call("sfx_transpose", rows, cols, px, ldx, out.data_ptr(), rows, stream())
    return out


def linear_bwd_data(dy: Tensor, weight_t: Tensor, *, rowscale: Optional[Tensor] = None, dact: int = DACT_NONE,
                    dact_ncols: int = -1, dact_pre: Optional[Tensor] = None, out: Optional[Tensor] = None,
                    accumulate: bool = False) -> Tensor:
    """dX = rowscale * (dY W) * act'(pre);  weight_t = W^T [K, N]."""
    M, N = dy.shape
    K = weight_t.shape[0]
    assert weight_t.shape[1] == N
    if out is None:
        assert not accumulate
        out = torch.empty(M, K, device=dy.device, dtype=torch.float32)
    pd, ldd = _rows(dy)
    pw, ldw = _rows(weight_t)
    po, ldo = _rows(out)
    pp, ldp = (None, 0) if dact_pre is None else _rows(dact_pre)
    call("sfx_linear_bwd_data", M, N, K, pd, ldd, pw, ldw, ptr(rowscale), dact, dact_ncols, pp, ldp, po, ldo,
         1 if accumulate else 0, *weight_split(weight_t), stream())
    return out


def linear_wgrad(dy: Tensor, x: Tensor, dw: Tensor, db: Optional[Tensor]) -> None:
    """dW += dY^T X ; db += colsum(dY)."""
    M, N = dy.shape
    K = x.shape[1]
    pd, ldd = _rows(dy)
    px, ldx = _rows(x)
    pw, ldw = _rows(dw)
    call("sfx_linear_wgrad", M, N, K, pd, ldd, px, ldx, pw, ldw, ptr(db), stream())


def subm_conv_bwd_data(dy: Tensor, smap, weight_t: Tensor, dx: Tensor) -> Tensor:
    """dx += SubMConv3d^T(dy) (accumulating)."""
    n, cout = dy.shape
    cin = dx.shape[1]
    pd, ldd = _rows(dy)
    px, ldx = _rows(dx)
    ws = torch.empty(2 * max(n, 1), device=dy.device, dtype=torch.int32)
    call("sfx_subm_conv_bwd_data", n, cin, cout, pd, ldd, ptr(smap.nbr), ptr(weight_t), ptr(smap.pair_in),
         ptr(smap.pair_out), smap._off_host, ws.data_ptr(), px, ldx, *weight_split(weight_t), stream())
    return dx


def window_attention_bwd(qkv: Tensor, order: Tensor, win: Tensor, num_windows: int, K: int, heads: int,
                         channels: int, dout: Tensor, attn_out: Optional[Tensor] = None) -> Tensor:
    """Backward of ptv3_ops.window_attention: query pass (dQ, per-query softmax statistics and dO.O from the
    forward output `attn_out`, recomputed here when not given) then key pass (dK, dV), attention.hip."""
    n = qkv.shape[0]
    if qkv.shape != (n, 3 * channels) or dout.shape != (n, channels) or tuple(win.shape) != (num_windows, 2):
        raise ValueError("window_attention_bwd: shape mismatch")
    if attn_out is None:
        from .ptv3_ops import window_attention
        attn_out = window_attention(qkv, order, win, num_windows, K, heads, channels)
    elif attn_out.shape != (n, channels) or not attn_out.is_contiguous():
        raise ValueError("window_attention_bwd: attn_out must be a contiguous [N, C] tensor")
    # the two-pass backward writes every element; the exact kernel (SFX_ATTN_PREC=fp32) accumulates into zeros
    dqkv = torch.zeros_like(qkv) if _ATTN_EXACT else torch.empty_like(qkv)
    stats = torch.empty(max(n, 1) * heads * 4, device=qkv.device, dtype=torch.float32)
    d = channels // heads
    call("sfx_window_attention_bwd", num_windows, K, heads, d, channels, ptr(qkv), ptr(order, torch.int32),
         ptr(win, torch.int32), float(d ** -0.5), ptr(attn_out), ptr(dout), ptr(dqkv), ptr(stats), stream())
    return dqkv


def window_attention_varlen_bwd(qkv: Tensor, order: Tensor, win3: Tensor, num_windows: int, K: int, heads: int,
                                channels: int, dout: Tensor) -> Tensor:
    """Backward of ptv3_ops.window_attention_varlen (enable_flash=True): query pass (dQ, per-query log-sum-exp and
    dO.O) then key pass (dK, dV), attention.hip."""
    n = qkv.shape[0]
    if qkv.shape != (n, 3 * channels) or dout.shape != (n, channels) or tuple(win3.shape) != (num_windows, 3):
        raise ValueError("window_attention_varlen_bwd: shape mismatch")
    dqkv = torch.zeros_like(qkv)
    stats = torch.empty(max(n, 1) * heads * 2, device=qkv.device, dtype=torch.float32)
    d = channels // heads
    call("sfx_window_attention_varlen_bwd", num_windows, K, heads, d, channels, ptr(qkv), ptr(order, torch.int32),
         ptr(win3, torch.int32), float(d ** -0.5), ptr(dout), ptr(dqkv), ptr(stats), stream())
    return dqkv


def layernorm_bwd(x: Tensor, gamma: Tensor, dy: Tensor, eps: float, dres: Optional[Tensor] = None,
                  out: Optional[Tensor] = None) -> Tensor:
    M, Cc = x.shape
    out = torch.empty(M, Cc, device=x.device, dtype=torch.float32) if out is None else out
    px, ldx = _rows(x)
    pd, ldd = _rows(dy)
    pr, ldr = (None, 0) if dres is None else _rows(dres)
    po, ldo = _rows(out)
    call("sfx_layernorm_bwd", M, Cc, px, ldx, ptr(gamma), pd, ldd, pr, ldr, float(eps), po, ldo, stream())
    return out


def cpe_ln_bwd(u: Tensor, x1: Tensor, g_cpe: Tensor, g1: Tensor, dx2: Tensor, dh: Tensor,
               eps: float) -> Tuple[Tensor, Tensor]:
    M, Cc = x1.shape
    dx1 = torch.empty_like(x1)
    du = torch.empty_like(u)
    call("sfx_cpe_ln_bwd", M, Cc, ptr(u), ptr(x1), ptr(g_cpe), ptr(g1), ptr(dx2), ptr(dh), float(eps), ptr(dx1),
         ptr(du), stream())
    return dx1, du


# ---- BatchNorm1d in train mode (+ GELU) ---------------------------------------------------------------
class BNState:
    """What the backward needs from a train-mode BN forward: input, batch mean/rstd, global row count
    (and the folded scale/shift, to apply the same normalisation again)."""
    __slots__ = ("x", "mean", "rstd", "count", "scale", "shift")

    def __init__(self, x, mean, rstd, count, scale, shift):
        self.x, self.mean, self.rstd, self.count, self.scale, self.shift = x, mean, rstd, count, scale, shift


def _colsum_ws(M: int, Cc: int, dev) -> Tuple[Tensor, int]:
    nbytes = int(_lib.fn("sfx_colsum2_workspace_bytes")(max(M, 1), Cc))
    return torch.empty(nbytes, device=dev, dtype=torch.uint8), nbytes


def _allreduce(t: Tensor, group) -> None:
    if group is not None:
        from .dist import allreduce_sum_
        allreduce_sum_(t, group)


def bn_train_forward(x: Tensor, bn: torch.nn.BatchNorm1d, act: int, residual: Optional[Tensor] = None,
                     residual_idx: Optional[Tensor] = None, out: Optional[Tensor] = None, group=None,
                     update_running: bool = True) -> Tuple[Tensor, BNState]:
    """y = act(BN_train(x)) (+ residual[residual_idx]); running stats updated in place (momentum 0.01).
    With `group` the statistics are SyncBatchNorm's (all-reduced sums and row counts)."""
    M, Cc = x.shape
    dev = x.device
    ws, nbytes = _colsum_ws(M, Cc, dev)
    sums = torch.empty(2 * Cc + 1, device=dev, dtype=torch.float64)
    px, ldx = _rows(x)
    call("sfx_bn_stats", M, Cc, px, ldx, ws.data_ptr(), nbytes, sums.data_ptr(), stream())
    count = float(M)
    if group is not None:
        sums[2 * Cc] = float(M)
        _allreduce(sums, group)
        count = float(sums[2 * Cc].item())
    mean = torch.empty(Cc, device=dev, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    scale = torch.empty_like(mean)
    shift = torch.empty_like(mean)
    rm = bn.running_mean if update_running else None
    rv = bn.running_var if update_running else None
    call("sfx_bn_finalize", Cc, count, sums.data_ptr(), ptr(bn.weight.detach()), ptr(bn.bias.detach()), float(bn.eps),
         float(bn.momentum), ptr(rm), ptr(rv), ptr(mean), ptr(rstd), ptr(scale), ptr(shift), stream())
    if update_running:
        # the kernel wrote the running stats through raw pointers: bump their versions so caches keyed
        # on (data_ptr, _version) -- ptv3.bn_affine's eval scale/shift -- see the new statistics
        torch.autograd.graph.increment_version(bn.running_mean)
        torch.autograd.graph.increment_version(bn.running_var)
        if bn.num_batches_tracked is not None:
            bn.num_batches_tracked.add_(1)
    if out is None:
        out = torch.empty(M, Cc, device=dev, dtype=torch.float32)
    po, ldo = _rows(out)
    pr, ldr = (None, 0) if residual is None else _rows(residual)
    call("sfx_affine_act", M, Cc, px, ldx, ptr(scale), ptr(shift), act, pr, ldr, ptr(residual_idx, torch.int32),
         po, ldo, stream())
    return out, BNState(x, mean, rstd, count, scale, shift)


def bn_apply(st: BNState, act: int, residual: Optional[Tensor] = None, residual_idx: Optional[Tensor] = None,
             out: Optional[Tensor] = None) -> Tensor:
    """act(x*scale + shift) (+ residual[residual_idx]) with the statistics of an earlier bn_train_forward."""
    x = st.x
    M, Cc = x.shape
    if out is None:
        out = torch.empty(M, Cc, device=x.device, dtype=torch.float32)
    px, ldx = _rows(x)
    po, ldo = _rows(out)
    pr, ldr = (None, 0) if residual is None else _rows(residual)
    call("sfx_affine_act", M, Cc, px, ldx, ptr(st.scale), ptr(st.shift), act, pr, ldr,
         ptr(residual_idx, torch.int32), po, ldo, stream())
    return out


def bn_act_bwd(st: BNState, bn: torch.nn.BatchNorm1d, act: int, dy: Tensor, out: Optional[Tensor] = None,
               accumulate: bool = False, group=None) -> Tensor:
    """d x of act(BN_train(x)) given dy (SyncBatchNorm sums all-reduced when `group` is set)."""
    x = st.x
    M, Cc = x.shape
    dev = x.device
    ws, nbytes = _colsum_ws(M, Cc, dev)
    sums = torch.empty(2 * Cc, device=dev, dtype=torch.float64)
    px, ldx = _rows(x)
    pd, ldd = _rows(dy)
    g, b = bn.weight.detach(), bn.bias.detach()
    call("sfx_bn_act_bwd_reduce", M, Cc, px, ldx, ptr(st.mean), ptr(st.rstd), ptr(g), ptr(b), act, pd, ldd,
         ws.data_ptr(), nbytes, sums.data_ptr(), stream())
    _allreduce(sums, group)
    if out is None:
        assert not accumulate
        out = torch.empty(M, Cc, device=dev, dtype=torch.float32)
    po, ldo = _rows(out)
    call("sfx_bn_act_bwd_apply", M, Cc, px, ldx, ptr(st.mean), ptr(st.rstd), ptr(g), ptr(b), act, pd, ldd,
         sums.data_ptr(), float(st.count), po, ldo, 1 if accumulate else 0, stream())
    return out


def segment_max_arg(x: Tensor, idx_ptr: Tensor, sidx: Tensor, m: int) -> Tuple[Tensor, Tensor]:
    Cc = x.shape[1]
    y = torch.empty(m, Cc, device=x.device, dtype=torch.float32)
    arg = torch.empty(m, Cc, device=x.device, dtype=torch.int32)
    call("sfx_segment_max_arg", m, Cc, ptr(idx_ptr, torch.int32), ptr(sidx, torch.int32), ptr(x), ptr(y), ptr(arg),
         stream())
    return y, arg


def segment_max_bwd(dy: Tensor, arg: Tensor, n_rows: int) -> Tensor:
    m, Cc = dy.shape
    dx = torch.zeros(n_rows, Cc, device=dy.device, dtype=torch.float32)
    call("sfx_segment_max_bwd", m, Cc, ptr(dy), ptr(arg, torch.int32), ptr(dx), stream())
    return dx


def segment_sum(x: Tensor, idx_ptr: Tensor, sidx: Tensor, m: int) -> Tensor:
    Cc = x.shape[1]
    px, ldx = _rows(x)
    y = torch.empty(m, Cc, device=x.device, dtype=torch.float32)
    call("sfx_segment_sum", m, Cc, ptr(idx_ptr, torch.int32), ptr(sidx, torch.int32), px, ldx, ptr(y), stream())
    return y


def act_bwd(dy: Tensor, pre: Tensor, act: int, ncols: int = -1, out: Optional[Tensor] = None) -> Tensor:
    M, N = dy.shape
    out = torch.empty(M, N, device=dy.device, dtype=torch.float32) if out is None else out
    pd, ldd = _rows(dy)
    pp, ldp = _rows(pre)
    po, ldo = _rows(out)
    call("sfx_act_bwd", M, N, pd, ldd, pp, ldp, act, N if ncols < 0 else ncols, po, ldo, stream())
    return out


def drop_mask(n: int, keep: float, seed: int, device) -> Tensor:
    """DropPath keep mask [n]: 1/keep with probability keep, else 0 (sfx_drop_mask, deterministic in seed)."""
    out = torch.empty(n, device=device, dtype=torch.float32)
    call("sfx_drop_mask", n, float(keep), seed & 0xFFFFFFFFFFFFFFFF, ptr(out), stream())
    return out


# ---- optimiser ------------------------------------------------------------------------------------------
def grad_clip_coef(grads, max_norm: float) -> Tuple[Tensor, Tensor]:
    """clip_grad_norm_ without a host sync: (coef [1] f32 on device, total norm [1] f32)."""
    dev = grads[0].device
    acc = torch.zeros(1, device=dev, dtype=torch.float64)
    for g in grads:
        call("sfx_sumsq", g.numel(), ptr(g), acc.data_ptr(), stream())
    coef = torch.empty(1, device=dev, dtype=torch.float32)
    norm = torch.empty(1, device=dev, dtype=torch.float32)
    call("sfx_clip_coef", acc.data_ptr(), float(max_norm), coef.data_ptr(), norm.data_ptr(), stream())
    return coef, norm


def adam_step(p: Tensor, g: Tensor, m1: Tensor, m2: Tensor, step: int, lr: float, betas=(0.9, 0.999),
              eps: float = 1e-8, weight_decay: float = 0.0, grad_scale: Optional[Tensor] = None) -> None:
    call("sfx_adam_step", p.numel(), ptr(p), ptr(g), ptr(m1), ptr(m2), ptr(grad_scale), float(lr), float(betas[0]),
         float(betas[1]), float(eps), float(weight_decay), int(step), stream())
