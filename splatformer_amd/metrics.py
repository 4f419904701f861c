"""Evaluation metrics on device: uint8-quantised PSNR and SSIM (reference utils/metrics.py + train.py:104-113).

`psnr_u8(pred, gt)` mirrors the reference evaluation contract for synthetic (3-channel) targets:
- train.py:104-113: `gt = (gt*255).to(uint8)`, `pred = (pred*255).to(uint8)` (truncation), pred having
  been clamped to <= 1 by gs_utils.py:111;
- utils/metrics.py:26-29: each batch is divided by 255 only if its max exceeds 1 (the max is taken over
  the whole [V,H,W,3] batch);
- utils/metrics.py:89-91: psnr = 20 log10(1 / sqrt(mse)) per image.

The quantisation and the per-image integer moments run in one HIP kernel (sfx_image_stats_u8); mse is
formed on the host from the exact integer sums.  Divergence (documented): when a batch's max is <= 1 and
the OTHER batch's is too, the reference subtracts two uint8 tensors (wrap-around) and then fails in
`.mean()` on a Byte tensor; here the values are used unscaled instead.
"""
from __future__ import annotations

import torch

import math

from . import _lib
from ._lib import I, L, P, Z, call, ptr, stream

_lib.register("sfx_image_stats_u8", [I, L, P, P, I, P, P, P])
_lib.register("sfx_ssim_workspace_bytes", [I, I, I, I], Z)
_lib.register("sfx_ssim", [I, I, I, I, P, P, P, I, P, P, Z, P])


def image_stats_u8(pred: torch.Tensor, gt: torch.Tensor, clamp_pred: bool = True):
    """Per-image exact integer moments of the quantised images: sums [V,3] (p², g², pg), maxes [V,2]."""
    _lib.require_gpu(pred)
    if pred.shape != gt.shape:
        raise ValueError(f"pred {tuple(pred.shape)} and gt {tuple(gt.shape)} differ")
    V = pred.shape[0]
    pred = pred.float().contiguous()
    gt = gt.float().contiguous()
    elems = pred.numel() // max(V, 1)
    sums = torch.empty(V, 3, device=pred.device, dtype=torch.int64)
    maxes = torch.empty(V, 2, device=pred.device, dtype=torch.int32)
    call("sfx_image_stats_u8", V, elems, ptr(pred), ptr(gt), 1 if clamp_pred else 0, ptr(sums), ptr(maxes),
         stream())
    return sums, maxes


def psnr_from_stats(sums: torch.Tensor, maxes: torch.Tensor, elems: int) -> torch.Tensor:
    """PSNR per image [V] (float64) from the integer moments and the batch-max scaling rule."""
    s = sums.to(torch.float64).cpu()
    m = maxes.cpu()
    a = 1.0 / 255.0 if int(m[:, 0].max()) > 1 else 1.0
    b = 1.0 / 255.0 if int(m[:, 1].max()) > 1 else 1.0
    sse = a * a * s[:, 0] + b * b * s[:, 1] - 2.0 * a * b * s[:, 2]
    mse = sse.clamp_min(0.0) / elems
    return 20.0 * torch.log10(1.0 / torch.sqrt(mse))


def psnr_u8(pred: torch.Tensor, gt: torch.Tensor, clamp_pred: bool = True) -> torch.Tensor:
    """[V,H,W,3] prediction and target in [0,1] -> per-image PSNR [V] (float64, on the host)."""
    sums, maxes = image_stats_u8(pred, gt, clamp_pred)
    return psnr_from_stats(sums, maxes, pred.numel() // max(pred.shape[0], 1))


def ssim_window(window_size: int = 11, sigma: float = 1.5) -> torch.Tensor:
    """The reference's 2-D window (metrics.py:93-101): normalised 1-D Gaussian (fp32), outer product."""
    g = torch.tensor([math.exp(-(x - window_size // 2) ** 2 / float(2 * sigma ** 2)) for x in range(window_size)],
                     dtype=torch.float32)
    g = (g / g.sum()).unsqueeze(1)
    return g.mm(g.t()).float()


_WIN = {}


def ssim(img1: torch.Tensor, img2: torch.Tensor, quantize_u8: bool = False) -> torch.Tensor:
    """[V,H,W,C] images (HWC) -> SSIM per image [V] (float32 on the device), = MetricComputer's
    `ssim(x.permute(0,3,1,2), ..., window_size=11, size_average=False)` (metrics.py:15, :103-135).
    quantize_u8: score the uint8 images of the evaluation loop (truncation, img1 clamped to <= 1, /255) --
    the batch-max rule of metrics.py:26-29 is taken as dividing (it differs only for images whose largest
    uint8 value is <= 1)."""
    _lib.require_gpu(img1)
    if img1.shape != img2.shape or img1.dim() != 4:
        raise ValueError(f"ssim: expected two equal [V,H,W,C] tensors, got {tuple(img1.shape)}, {tuple(img2.shape)}")
    V, H, W, C = img1.shape
    a = img1.float().contiguous()
    b = img2.float().contiguous()
    dev = a.device
    win = _WIN.get(dev)
    if win is None:
        win = _WIN[dev] = ssim_window().reshape(-1).to(dev)
    nbytes = _lib.fn("sfx_ssim_workspace_bytes")(V, H, W, C)
    ws = torch.empty(max(int(nbytes), 4), dtype=torch.uint8, device=dev)
    out = torch.empty(V, dtype=torch.float32, device=dev)
    call("sfx_ssim", V, H, W, C, ptr(a), ptr(b), ptr(win), 1 if quantize_u8 else 0, ptr(out), ptr(ws), ws.numel(),
         stream())
    return out

