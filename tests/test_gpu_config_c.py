"""Config C at its own workload: the training step the C bench line times, compared with
the CPU oracle at full size -- one 100k-Gaussian SH1 scene exactly as bench.py --config C builds it (scene seed
0, duplicate voxels kept, ptv3_base weights from torch.manual_seed(0)), 4 training views at 800x800, the
synthetic targets = renders of the input scene.

The step is reference train.py:236-289: train-mode refine (batch-statistics BatchNorm, DropPath), render of the
refined Gaussians through the reference glue (gs_utils.py:29-112) on the gsplat-v0.1.11 autograd ops, image-L1
loss (train.py:272-286, / num_images / len(batch)), backward through renderer and refiner to the attn.qkv
parameters (utils/optimizers.py:48-52).  Checked against the oracle:

* forward: the refined residual of the train-mode refine, relative L2 <= 1e-5 (same weights, the same five
  order shuffles and DropPath masks, recorded from the HIP run and replayed);
* render backward, every view: the rasterizer's v_xy / v_conic / v_rgb / v_opacity for the upstream gradient
  HIP's loss produced (gsplat_ref.rasterize_backward on the HIP rasterizer's own inputs) and the projection's
  v_mean / v_scale / v_quat (gsplat_ref.project_gaussians_backward): max |diff| <= 2e-4 of the largest
  magnitude and relative L2 <= 2e-4;
* refiner backward: the qkv gradients for HIP's d(loss)/d(refined record), as close to the fp64 oracle as the
  fp32 oracle is (2x + 1e-5; the bar of tests/test_gpu_train.py, with the heads' ReLU active sets replayed).

Reference-precision mode (Trainer(precision="amp") = the reference's `training.enable_amp`, train.py:240,
configs/train/default.gin:11; ops.precision / include/sfx.h sfx_set_precision): the same train-mode refine and
refiner backward (same weights, order shuffles, DropPath masks and upstream gradient) in that mode, against the
oracle in its autocast mode (oracle/ptv3_ref.autocast: every value CUDA autocast holds in fp16 rounded to fp16;
the reference's GradScaler loss scaling emulated):
the refined residual's distance to the fp32 oracle and the qkv gradients' distance to the fp32 oracle run on the amp
run's head ReLU active sets are at most 1.5x the autocast oracle's own (the autocast oracle replays the same active
sets, so neither side carries ReLU-flip error and the bar measures the fp16 rounding, ~1e-3); the residual
measurably differs from the fp32 mode's (> 1e-5: the mode is on).
"""
import pytest
import torch

from oracle import gsplat_ref, ptv3_ref
from splatformer_amd import gs_render
from splatformer_amd import ptv3_ops as ops
from splatformer_amd import train as strain
from splatformer_amd.scenes import make_cameras, make_scene, to_device
from test_gpu_ptv3 import rel_l2
from test_gpu_train import FEATS, RecordingMasks

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

N, RES, VIEWS = 100_000, 800, 4


@pytest.fixture(scope="module")
def hip_c(device):
    from _pytest.monkeypatch import MonkeyPatch
    from splatformer_amd.feature_predictor import FeaturePredictor
    torch.manual_seed(0)
    model = FeaturePredictor(sh_degree=1, zeroinit=False)
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}  # before the train forward moves BN stats
    model = model.to(device)
    for name, p in model.named_parameters():
        p.requires_grad_("attn.qkv" in name)
        p.grad = torch.zeros_like(p) if p.requires_grad else None
    scene = make_scene(N, 1, seed=0)
    gs = to_device(scene, device)
    cams = to_device(make_cameras(RES, RES, n_views=VIEWS), device)
    with torch.no_grad():
        gts = gs_render.rasterize_gaussians_to_multiimgs(gs, cams)[0]
    masks = RecordingMasks(77)
    torch.manual_seed(1)
    packed, tape = strain.refine_train(model, gs, masks)
    perms = model.backbone.backbone.last_perms
    W = model.width
    relu = {f: [(h[:, g * W:(g + 1) * W] > 0).cpu() for h in tape["hs"]] for g, f in enumerate(model.output_features)}
    leaf, out_gs = strain.unpack_leaf(model, packed, gs)

    views = []
    orig_p, orig_r = gs_render.project_gaussians, gs_render.rasterize_gaussians

    def cap_project(means, scales, glob_scale, quats, viewmat, *rest):
        # per-view identity nodes: the glue's inputs are shared by the views, their per-view gradients are not
        m, s, q = means.view_as(means), scales.view_as(scales), quats.view_as(quats)
        for t in (m, s, q):
            t.retain_grad()
        out = orig_p(m, s, glob_scale, q, viewmat, *rest)
        views.append(dict(proj_in=(m, s, q), viewmat=viewmat.detach().cpu(), proj_out=out))
        return out

    def cap_raster(xys, depths, radii, conics, num_tiles_hit, colors, opacity, img_height, img_width, block_width,
                   background=None, return_alpha=False):
        opacity = opacity.view_as(opacity)  # per-view node: the activated opacities are shared by the views
        for t in (xys, conics, colors, opacity):
            t.retain_grad()
        rgb, alpha = orig_r(xys, depths, radii, conics, num_tiles_hit, colors, opacity, img_height, img_width,
                            block_width, background=background, return_alpha=return_alpha)
        rgb.retain_grad()
        views[-1].update(r_in=(xys, depths, radii, conics, num_tiles_hit, colors, opacity), rgb=rgb, bg=background)
        return rgb, alpha

    mp = MonkeyPatch()
    mp.setattr(gs_render, "project_gaussians", cap_project)
    mp.setattr(gs_render, "rasterize_gaussians", cap_raster)
    try:
        with torch.enable_grad():
            preds, _ = gs_render.rasterize_gaussians_to_multiimgs(out_gs, cams)
            loss = strain.image_l1(preds, gts) / VIEWS / 1
            loss.backward()
    finally:
        mp.undo()
    d_packed = leaf.grad.detach().clone()
    strain.refine_backward(model, tape, d_packed)
    torch.cuda.synchronize()
    cpu = lambda t: t.detach().cpu()
    vcap = []
    for v in views:
        xys, depths, radii, conics, tiles, colors, opac = v["r_in"]
        m, s, q = v["proj_in"]
        out = v["proj_out"]
        vcap.append(dict(
            r_in=[cpu(t) for t in (xys, depths, radii, conics, tiles, colors, opac)], bg=cpu(v["bg"]),
            v_out=cpu(v["rgb"].grad), r_grad=[cpu(t.grad) for t in (xys, conics, colors, opac)],
            p_in=[cpu(t) for t in (m, s, q)], p_grad=[cpu(t.grad) for t in (m, s, q)], viewmat=v["viewmat"],
            cov3d=cpu(out[6]), comp=cpu(out[4])))
    mpar = dict(model.named_parameters())
    names = [k for k in sd if "attn.qkv" in k]
    return dict(sd=sd, scene=scene, perms=perms, masks=masks.masks, relu=relu, packed=cpu(packed),
                d_packed=cpu(d_packed), views=vcap, cams=make_cameras(RES, RES, n_views=VIEWS),
                grads={k: cpu(mpar[k].grad) for k in names}, names=names, loss=float(loss.detach()))


def _oracle(hip, dtype, autocast=False, relu=None):
    """Oracle train-mode refine + autograd to the qkv parameters for HIP's upstream gradient, in `dtype`.
    autocast=True: in the reference's autocast precision with its GradScaler (train.py:215, :289-299: the loss
    scaled by 2^16, halved after a step whose gradients overflow, gradients unscaled before use) -- without the
    scaling the fp16 gradients underflow and the oracle's qkv gradients are noise."""
    scale = 65536.0 if autocast else 1.0
    while True:
        sd = {k: (v.to(dtype) if v.is_floating_point() else v).clone() for k, v in hip["sd"].items()}
        for k in hip["names"]:
            sd[k].requires_grad_()
        sc = {k: v.to(dtype) for k, v in hip["scene"].items()}
        mk = {k: m.to(dtype) for k, m in hip["masks"].items()}
        with ptv3_ref.autocast(autocast):
            ref, _ = ptv3_ref.feature_predictor_forward(sd, ptv3_ref.PTv3Config(), sc, hip["perms"], train=True,
                                                        masks=mk, relu_masks=relu or hip["relu"])
            rp = torch.cat([ref[f].reshape(N, -1) for f in FEATS], 1)
            (rp * (hip["d_packed"].to(dtype) * scale)).sum().backward()
        grads = {k: sd[k].grad.double() / scale for k in hip["names"]}
        if all(torch.isfinite(g).all() for g in grads.values()) or scale <= 1.0:
            return grads, rp.detach()
        scale /= 2.0


@pytest.fixture(scope="module")
def oracle32(hip_c):
    return _oracle(hip_c, torch.float32)


@pytest.fixture(scope="module")
def oracle64(hip_c):
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        g64, _ = _oracle(hip_c, torch.float64)
    finally:
        torch.set_default_dtype(prev)
    return g64


def test_config_c_train_forward(hip_c, oracle32):
    _, ref_packed = oracle32
    s = hip_c["scene"]
    in_packed = torch.cat([s[f].reshape(N, -1) for f in FEATS], 1)
    err = rel_l2(hip_c["packed"] - in_packed, ref_packed - in_packed)
    print(f"\n[config C] train-forward residual rel L2 {err:.2e}, loss {hip_c['loss']:.6f}")
    assert err < 1e-5


def _close(got, exp, nm, bar=2e-4):
    scale = exp.abs().max().clamp_min(1e-12)
    e_max = float((got - exp).abs().max() / scale)
    e_l2 = rel_l2(got, exp)
    assert e_max < bar and e_l2 < bar, f"{nm}: max-rel {e_max:.2e}, rel L2 {e_l2:.2e}"
    return e_max


@pytest.mark.parametrize("v", range(VIEWS))
def test_config_c_render_backward(hip_c, v):
    c = hip_c["views"][v]
    xys, depths, radii, conics, tiles, colors, opac = c["r_in"]
    H = W = RES
    tx, ty = (W + 15) // 16, (H + 15) // 16
    _, gids, bins = gsplat_ref.bin_and_sort_gaussians(xys, depths, radii, tiles, tx, ty, 16)
    img, fT, fidx = gsplat_ref.rasterize_forward(tx, ty, 16, H, W, gids, bins, xys, conics, colors, opac, c["bg"])
    v_alpha = torch.zeros(H, W)  # the L1 loss reads the image only
    ref = gsplat_ref.rasterize_backward(tx, ty, 16, H, W, gids, bins, xys, conics, colors, opac, c["bg"], fT, fidx,
                                        c["v_out"], v_alpha)
    errs = [_close(g, e, nm) for nm, g, e in zip(["v_xy", "v_conic", "v_rgb", "v_opacity"], c["r_grad"], ref)]
    # projection backward for the rasterizer's v_xy / v_conic (v_depth, v_comp do not reach the loss)
    m, s, q = c["p_in"]
    cams = hip_c["cams"]
    n = m.shape[0]
    pref = gsplat_ref.project_gaussians_backward(m, s, 1.0, q, c["viewmat"], float(cams["fx"]), float(cams["fy"]),
                                                 c["cov3d"], radii, conics, c["comp"], c["r_grad"][0], torch.zeros(n),
                                                 c["r_grad"][1], torch.zeros(n))
    errs += [_close(g, e, nm, 1e-4) for nm, g, e in zip(["v_mean", "v_scale", "v_quat"], c["p_grad"], pref)]
    print(f"\n[config C view {v}] raster/project backward max-rel errors {['%.1e' % e for e in errs]}")


def test_config_c_qkv_grads(hip_c, oracle32, oracle64):
    g32, _ = oracle32
    g64 = oracle64
    names = hip_c["names"]
    hip = torch.cat([hip_c["grads"][k].double().reshape(-1) for k in names])
    r32 = torch.cat([g32[k].reshape(-1) for k in names])
    r64 = torch.cat([g64[k].reshape(-1) for k in names])
    e_hip, e_ref = rel_l2(hip, r64), rel_l2(r32, r64)
    print(f"\n[config C] qkv grads to fp64: HIP {e_hip:.2e}, fp32 oracle {e_ref:.2e}")
    assert e_hip <= 2.0 * e_ref + 1e-5


# ---- reference-precision mode ---------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def hip_amp(device, hip_c):
    """The train-mode refine + refiner backward of hip_c in precision "amp", for hip_c's upstream gradient."""
    from splatformer_amd.feature_predictor import FeaturePredictor
    torch.manual_seed(0)
    model = FeaturePredictor(sh_degree=1, zeroinit=False).to(device)
    for name, p in model.named_parameters():
        p.requires_grad_("attn.qkv" in name)
        p.grad = torch.zeros_like(p) if p.requires_grad else None
    gs = to_device(hip_c["scene"], device)
    masks = RecordingMasks(77)
    torch.manual_seed(1)
    with ops.precision("amp"):
        packed, tape = strain.refine_train(model, gs, masks)
        W = model.width
        relu = {f: [(h[:, g * W:(g + 1) * W] > 0).cpu() for h in tape["hs"]]
                for g, f in enumerate(model.output_features)}
        strain.refine_backward(model, tape, hip_c["d_packed"].to(device))
    torch.cuda.synchronize()
    # the same order shuffles and DropPath masks as the fp32 run (so the oracle runs of hip_c apply)
    assert model.backbone.backbone.last_perms == hip_c["perms"]
    assert all(torch.equal(masks.masks[k], hip_c["masks"][k]) for k in hip_c["masks"])
    mpar = dict(model.named_parameters())
    return dict(packed=packed.detach().cpu(), grads={k: mpar[k].grad.detach().cpu() for k in hip_c["names"]},
                relu=relu)


# The autocast oracle replays the HIP amp run's head ReLU active sets: a unit whose pre-activation lies within the
# amp rounding of 0 flips between the precisions, and both amp-side gradients then carry the same flips against
# the fp64 reference (which keeps the fp32 run's sets).
@pytest.fixture(scope="module")
def oracle_amp(hip_c, hip_amp):
    return _oracle(hip_c, torch.float32, autocast=True, relu=hip_amp["relu"])


def test_config_c_amp_train_forward(hip_c, hip_amp, oracle32, oracle_amp):
    _, ref32 = oracle32
    _, ref16 = oracle_amp
    s = hip_c["scene"]
    inp = torch.cat([s[f].reshape(N, -1) for f in FEATS], 1)
    e_hip = rel_l2(hip_amp["packed"] - inp, ref32 - inp)
    e_orc = rel_l2(ref16 - inp, ref32 - inp)
    print(f"\n[config C amp] train-forward residual rel L2 to the fp32 oracle: HIP amp {e_hip:.2e}, "
          f"autocast oracle {e_orc:.2e}")
    assert 1e-5 < e_hip <= 1.5 * e_orc


@pytest.fixture(scope="module")
def oracle32_amp_relu(hip_c, hip_amp):
    """The fp32 oracle on the amp run's head ReLU active sets: the reference the amp-side qkv gradients are held to.
    Against the fp64 oracle (the fp32 run's active sets) both amp sides carry the same ~1e-2 of ReLU flips, which
    would hide ~1e-2 of extra amp-path error under a 1.5x bar; with the flips replayed on the reference side the
    distance measured is the fp16 rounding itself (~1e-3)."""
    return _oracle(hip_c, torch.float32, relu=hip_amp["relu"])[0]


def test_config_c_amp_qkv_grads(hip_c, hip_amp, oracle_amp, oracle32_amp_relu):
    g16, _ = oracle_amp
    names = hip_c["names"]
    hip = torch.cat([hip_amp["grads"][k].double().reshape(-1) for k in names])
    r16 = torch.cat([g16[k].reshape(-1) for k in names])
    r32 = torch.cat([oracle32_amp_relu[k].double().reshape(-1) for k in names])
    e_hip, e_orc = rel_l2(hip, r32), rel_l2(r16, r32)
    print(f"\n[config C amp] qkv grads to the fp32 oracle on the amp ReLU sets: HIP amp {e_hip:.2e}, "
          f"autocast oracle {e_orc:.2e}")
    assert e_orc < 1e-2  # the reference carries no ReLU-flip error: the bar measures fp16 rounding
    assert e_hip <= 1.5 * e_orc
