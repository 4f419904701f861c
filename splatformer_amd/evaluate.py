"""Evaluation loop of the hot path (reference train.py:76-176 `evaluation`, test branch).

For each scene of this rank's chunk (dataset/GS.py:54-67): refine with the FeaturePredictor (one scene
per forward, feature_predictor.py:244), render the V test views of the refined Gaussians
(gs_utils.rasterize_gaussians_to_multiimgs), quantise prediction and target to uint8 and accumulate the
per-image PSNR and SSIM sums (train.py:104-131, utils/metrics.py); finally reduce to rank 0
(train.py:170-176).  LPIPS (VGG weights, unavailable offline) is out of scope.
"""
from __future__ import annotations

from typing import Callable, Dict, Sequence

import torch

from . import _lib, dist
from .gs_render import rasterize_gaussians_to_multiimgs
from .metrics import image_stats_u8, psnr_from_stats, ssim


@torch.no_grad()
def evaluate_scenes(model, scenes: Sequence[dict], cameras: Sequence[dict],
                    targets: Callable[[int], torch.Tensor], device: torch.device,
                    evaluate_input: bool = False) -> Dict[str, float]:
    """Evaluate this rank's chunk of `scenes`.

    scenes[i]: normalized Gaussian dict (device tensors); cameras[i]: camera dict (device tensors);
    targets(i): [V,H,W,3] ground-truth images in [0,1] for scene i (device).
    Returns the rank-0 reduced means ({} on other ranks)."""
    rank, ws = dist.world()
    mine = dist.scene_chunk(len(scenes), rank, ws)
    psnr_sum = torch.zeros((), dtype=torch.float64)
    ssim_sum = torch.zeros((), dtype=torch.float64)
    num_images = 0
    for i in mine:
        gs = scenes[i] if evaluate_input else model([scenes[i]], [i])[0]
        rgbs, _ = rasterize_gaussians_to_multiimgs(gs, cameras[i])
        pred = torch.stack(rgbs, 0)
        gt = targets(i)
        sums, maxes = image_stats_u8(pred, gt, clamp_pred=False)  # rgbs are already clamped (gs_utils.py:111)
        psnr = psnr_from_stats(sums, maxes, pred[0].numel())
        psnr_sum += psnr.sum()
        ssim_sum += ssim(pred, gt, quantize_u8=True).double().sum().cpu()
        num_images += pred.shape[0]
        if not evaluate_input and hasattr(model, "check_refine"):
            model.check_refine()  # the refine's deferred pooling checks, at the readback that consumes it
        else:
            _lib.check_lookback("evaluate_scenes")  # the render's intersection scans / sorts
    return dist.reduce_metrics({"psnr": psnr_sum, "ssim": ssim_sum}, num_images, len(mine),
                               device=device if ws > 1 and device.type == "cuda" else None)
