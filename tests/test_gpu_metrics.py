"""HIP uint8 PSNR (sfx_image_stats_u8) vs the oracle restatement of train.py:104-113 + utils/metrics.py.

Tolerance: |dPSNR| <= 1e-4 dB (BASELINE.json north_star); the HIP side is exact integer moments, the
oracle a float32 mean, so the difference is the oracle's rounding."""
import pytest
import torch

from oracle import gsplat_ref
from splatformer_amd import metrics
from splatformer_amd.evaluate import evaluate_scenes
from splatformer_amd.scenes import make_cameras, make_scene, to_device

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(3, 64, 48, 3), (9, 200, 200, 3), (1, 1, 1, 3)])
def test_psnr_u8_matches_oracle(device, shape):
    g = torch.Generator().manual_seed(shape[1])
    gt = torch.rand(shape, generator=g)
    pred = (gt + 0.05 * torch.randn(shape, generator=g)).clamp_min(0) * 1.02  # some values > 1
    want = gsplat_ref.psnr_u8(pred.clamp(max=1.0), gt).reshape(-1).double()
    got = metrics.psnr_u8(pred.to(device), gt.to(device))
    assert torch.allclose(got, want, atol=1e-4, rtol=0)


def test_psnr_u8_max_rule(device):
    # a target batch whose quantised max is 1 is NOT divided by 255 (metrics.py:26-29)
    gt = torch.full((2, 8, 8, 3), 1.5 / 255)
    pred = torch.rand(2, 8, 8, 3, generator=torch.Generator().manual_seed(0))
    want = gsplat_ref.psnr_u8(pred, gt).reshape(-1).double()
    got = metrics.psnr_u8(pred.to(device), gt.to(device))
    assert torch.allclose(got, want, atol=1e-4, rtol=0)


def test_identical_images_give_inf(device):
    x = torch.rand(2, 16, 16, 3, device=device)
    assert torch.isinf(metrics.psnr_u8(x, x)).all()


def test_evaluate_scenes_single_rank(device):
    """evaluate_input=True (train.py:96-97 branch) keeps the check deterministic: the refiner's
    order shuffle draws from the global RNG on every forward."""
    from splatformer_amd.feature_predictor import FeaturePredictor
    from splatformer_amd.gs_render import rasterize_gaussians_to_multiimgs
    torch.manual_seed(0)
    model = FeaturePredictor(sh_degree=1, zeroinit=False).eval().to(device)
    scenes = [to_device(make_scene(3000, sh_degree=1, seed=s), device) for s in range(2)]
    cams = [to_device(make_cameras(64, 64, n_views=3), device) for _ in range(2)]
    noise = torch.Generator().manual_seed(1)
    renders, targets = [], []
    for s in range(2):
        with torch.no_grad():
            rgbs, _ = rasterize_gaussians_to_multiimgs(scenes[s], cams[s])
        r = torch.stack(rgbs, 0).cpu()
        renders.append(r)
        targets.append((r + 0.02 * torch.rand(3, 64, 64, 3, generator=noise)).clamp(0, 1))
    got = evaluate_scenes(model, scenes, cams, lambda i: targets[i].to(device), device, evaluate_input=True)
    want = torch.cat([gsplat_ref.psnr_u8(renders[s], targets[s]).reshape(-1) for s in range(2)])
    assert got["num_images"] == 6 and got["num_scenes"] == 2
    assert got["psnr"] == pytest.approx(float(want.double().mean()), abs=1e-4)
    # SSIM of the uint8 images /255 (train.py:104-113 -> metrics.py:26-29, :103-135)
    from oracle import metrics_ref
    q = lambda x: (x * 255).to(torch.uint8).float().div(255.0).permute(0, 3, 1, 2)  # noqa: E731
    want_ssim = torch.cat([metrics_ref.ssim(q(renders[s].clamp(max=1)), q(targets[s]), 11, size_average=False)
                           for s in range(2)])
    assert got["ssim"] == pytest.approx(float(want_ssim.double().mean()), abs=2e-6)
    refined = evaluate_scenes(model, scenes, cams, lambda i: targets[i].to(device), device)
    assert refined["num_images"] == 6 and refined["psnr"] == refined["psnr"]  # finite / not NaN


def test_ssim_matches_reference_golden(device):
    """sfx_ssim vs the outputs of the reference's own utils/metrics.py ssim (tests/golden/metrics.npz) and the
    oracle on a render-sized batch (HWC layout as rendered; tolerance 2e-6 absolute on an SSIM in [-1, 1])."""
    import os
    import numpy as np
    from oracle import metrics_ref
    from splatformer_amd import metrics
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "metrics.npz"))
    for i in range(2):
        a, b = torch.from_numpy(d[f"b{i}_img1"]), torch.from_numpy(d[f"b{i}_img2"])
        got = metrics.ssim(a.permute(0, 2, 3, 1).to(device), b.permute(0, 2, 3, 1).to(device)).cpu()
        assert (got - torch.from_numpy(d[f"b{i}_ssim"])).abs().max() < 2e-6
    g = torch.Generator().manual_seed(3)
    x = torch.rand(3, 130, 97, 3, generator=g)
    y = (x + 0.05 * torch.randn(x.shape, generator=g)).clamp(0, 1)
    ref = metrics_ref.ssim(x.permute(0, 3, 1, 2), y.permute(0, 3, 1, 2), 11, size_average=False)
    got = metrics.ssim(x.to(device), y.to(device)).cpu()
    assert (got - ref).abs().max() < 2e-6
