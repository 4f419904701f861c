"""CPU restatement of the reference evaluation metrics (utils/metrics.py:86-135).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Pinned by tests/golden/metrics.npz, captured from the
reference's own utils/metrics.py (tests/golden/make_golden.py part 4).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def psnr(img1, img2):
    """metrics.py:89-91 on [N,...] batches."""
    mse = ((img1 - img2) ** 2).view(img1.shape[0], -1).mean(1, keepdim=True)
    return 20 * torch.log10(1.0 / torch.sqrt(mse))


def _window(window_size, channel):
    """metrics.py:93-101."""
    g = torch.tensor([math.exp(-(x - window_size // 2) ** 2 / float(2 * 1.5 ** 2)) for x in range(window_size)],
                     dtype=torch.float32)
    g = (g / g.sum()).unsqueeze(1)
    w2 = g.mm(g.t()).float().unsqueeze(0).unsqueeze(0)
    return w2.expand(channel, 1, window_size, window_size).contiguous()


def ssim(img1, img2, window_size=11, size_average=True):
    """metrics.py:103-135 on NCHW batches; size_average=False -> per-image means [N]."""
    channel = img1.size(-3)
    w = _window(window_size, channel).type_as(img1)
    pad = window_size // 2
    mu1 = F.conv2d(img1, w, padding=pad, groups=channel)
    mu2 = F.conv2d(img2, w, padding=pad, groups=channel)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1 = F.conv2d(img1 * img1, w, padding=pad, groups=channel) - mu1_sq
    s2 = F.conv2d(img2 * img2, w, padding=pad, groups=channel) - mu2_sq
    s12 = F.conv2d(img1 * img2, w, padding=pad, groups=channel) - mu1_mu2
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    m = ((2 * mu1_mu2 + C1) * (2 * s12 + C2)) / ((mu1_sq + mu2_sq + C1) * (s1 + s2 + C2))
    return m.mean() if size_average else m.mean(1).mean(1).mean(1)
