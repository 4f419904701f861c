"""Oracle render glue vs golden vectors captured from the reference's own gs_utils.py
(tests/golden/make_golden.py).  Pins utils/gs_utils.py:31-95 argument semantics."""
import os

import numpy as np
import pytest
import torch

from oracle import gsplat_ref, render_ref

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "render_glue.npz")


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD))


@pytest.mark.parametrize("deg", [0, 1, 3])
def test_glue_args_match_reference(gold, deg):
    p = f"deg{deg}_"
    s = {k[len(p) + 3:]: torch.from_numpy(v) for k, v in gold.items() if k.startswith(p + "in_")}
    c2w = torch.from_numpy(gold[p + "c2w"])
    a = render_ref.glue_args(s, c2w)
    np.testing.assert_array_equal(a["viewmat"].numpy(), gold[p + "viewmat"])
    np.testing.assert_array_equal(a["scales"].numpy(), gold[p + "scales"])
    np.testing.assert_array_equal(a["quats"].numpy(), gold[p + "quats"])
    np.testing.assert_array_equal(a["opacities"].numpy(), gold[p + "opacity"])
    np.testing.assert_allclose(a["rgbs"].numpy(), gold[p + "colors"], rtol=0, atol=0)
    sc = gold[p + "proj_scalars"]
    assert sc[0] == 1 and sc[7] == 16  # glob_scale=1, BLOCK_WIDTH=16 (gs_utils.py:12, :85)
    intr = gold[p + "intr"]
    assert sc[5] == intr[5] and sc[6] == intr[4]  # H, W from height/width
    if deg > 0:
        assert int(gold[p + "sh_deg"]) == deg
        np.testing.assert_array_equal(a["viewdirs"].numpy(), gold[p + "sh_viewdirs"])
        np.testing.assert_array_equal(a["colors"].numpy(), gold[p + "sh_coeffs"])


def test_nan_quaternion_patched(gold):
    q = gold["deg1_quats"]
    np.testing.assert_array_equal(q[5], np.array([0, 0, 0, 1], dtype=np.float32))
    assert np.isfinite(q).all()


def test_metrics_oracle_matches_reference_golden():
    """oracle/metrics_ref.py (psnr, ssim) against outputs of the reference's own utils/metrics.py."""
    from oracle import metrics_ref
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "metrics.npz"))
    for i in range(2):
        a, b = torch.from_numpy(d[f"b{i}_img1"]), torch.from_numpy(d[f"b{i}_img2"])
        np.testing.assert_array_equal(metrics_ref.ssim(a, b, 11, size_average=False).numpy(), d[f"b{i}_ssim"])
        np.testing.assert_array_equal(metrics_ref.psnr(a, b).numpy(), d[f"b{i}_psnr"])
