"""Capture golden vectors from the reference's own glue code (run in the build
container only; /root/reference does not exist on the GPU box).

The reference's Python glue imports with stub modules for its absent
dependencies (gin, cv2, plyfile, torch_scatter, gsplat, pointcept), see
SURVEY.md §8(c).  We then run:

1. `utils/gs_utils.py:rasterize_gaussians_to_singleimg` with a *recording*
   gsplat stub: the arguments the glue hands to gsplat (viewmat, exp'd
   scales, normalised/NaN-patched quats, sigmoid opacities, SH coeff layout,
   viewdirs, clamp(+0.5) colours, H/W/fx/fy/cx/cy/block width, background)
   are saved -- they pin the render glue (oracle/render_ref.py and the fused
   HIP prep kernel).
2. `models/feature_predictor.py:FeaturePredictor` (ptv3_base.gin head config,
   zeroinit off so heads are non-trivial) with a recording stub backbone:
   the backbone input dict (coord, grid_coord, offset, feat) and the refined
   outputs for a fixed backbone feature pin batchify / grid_coord / heads /
   residual / tanh semantics.

3. `dataset/GS.py:SplatfactoDataset` scene loading (load_gs_params_fromnerfstudio,
   load_images_cameras_fromnerfstudio, load_scene, read_image) on a synthetic
   nerfstudio/colmap directory written here (NaN rows, inf scales, outliers,
   more than max_gs_num Gaussians, elevation-named OOD test views, an RGBA
   image): pins splatformer_amd/scene_io.py.

Outputs: tests/golden/render_glue.npz, tests/golden/feature_predictor.npz,
tests/golden/scene_io.npz, tests/golden/metrics.npz (inputs and outputs only -- data, no reference source).

4. `utils/metrics.py` psnr / ssim (lpips stubbed: its VGG weights are not available offline) on seeded image
   batches: pins oracle/metrics_ref.py and the SSIM kernel.
5. `utils/gs_utils.py` export_ply_forviewer (plyfile stubbed to record the vertex array) for SH degree 1 and 0
   scenes and prepare_viewer (cfg_args, cameras.json): pins splatformer_amd/export.py (tests/golden/export.npz).
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def install_stubs(recorder):
    gin = types.ModuleType("gin")

    def configurable(*a, **k):
        if a and callable(a[0]):
            return a[0]
        return lambda f: f

    gin.configurable = configurable
    gin.external_configurable = lambda *a, **k: a[0]
    gin.query_parameter = lambda name: recorder.get("gin", {}).get(name)
    sys.modules["gin"] = gin
    for m in ["cv2", "torch_scatter", "lpips"]:
        sys.modules[m] = types.ModuleType(m)
    ply = types.ModuleType("plyfile")

    class PlyElement:  # records the vertex array export_ply_forviewer builds
        @staticmethod
        def describe(elements, name):
            recorder["ply_elements"] = elements.copy()
            return (name, elements)

    class PlyData:
        def __init__(self, els):
            self.els = els

        def write(self, path):
            recorder["ply_path"] = path

    ply.PlyData = PlyData
    ply.PlyElement = PlyElement
    sys.modules["plyfile"] = ply

    gs = types.ModuleType("gsplat")

    def spherical_harmonics(deg, viewdirs, coeffs):
        recorder["sh"] = dict(deg=deg, viewdirs=viewdirs.clone(), coeffs=coeffs.clone())
        from oracle import gsplat_ref
        return gsplat_ref.spherical_harmonics(deg, viewdirs, coeffs)

    def project_gaussians(*args):
        names = ["means3d", "scales", "glob_scale", "quats", "viewmat", "fx", "fy", "cx", "cy", "img_height",
                 "img_width", "block_width"]
        recorder["project"] = {k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in zip(names, args)}
        from oracle import gsplat_ref
        return gsplat_ref.project_gaussians(*args)

    def rasterize_gaussians(xys, depths, radii, conics, num_tiles_hit, colors, opacity, H, W, bw, background=None,
                            return_alpha=False):
        recorder["raster"] = dict(colors=colors.clone(), opacity=opacity.clone(), H=H, W=W, bw=bw,
                                  background=background.clone(), return_alpha=return_alpha)
        from oracle import gsplat_ref
        return gsplat_ref.rasterize_gaussians(xys, depths, radii, conics, num_tiles_hit, colors, opacity, H, W, bw,
                                              background=background, return_alpha=return_alpha)

    gs.spherical_harmonics = spherical_harmonics
    gs.project_gaussians = project_gaussians
    gs.rasterize_gaussians = rasterize_gaussians
    sys.modules["gsplat"] = gs

    # reference models/pointtransformer_v3.py needs pointcept/spconv: stub the module with a recording backbone
    ptv3 = types.ModuleType("models.pointtransformer_v3")

    class PointTransformerV3Model(torch.nn.Module):
        output_dim = 96

        def __init__(self, in_channels, additional_info=None, **kw):
            super().__init__()
            g = torch.Generator().manual_seed(1234)
            self.proj = torch.nn.Parameter(torch.randn(in_channels + 3, 96, generator=g) * 0.3)

        def forward(self, data_dict):
            recorder["backbone_in"] = {k: (v.clone() if isinstance(v, torch.Tensor) else v)
                                       for k, v in data_dict.items()}
            x = torch.cat([data_dict["feat"], data_dict["grid_coord"].float() / 384.0], 1)
            feat = torch.tanh(x @ self.proj)
            recorder["backbone_out"] = feat.clone()
            return {"feat": feat}

    ptv3.PointTransformerV3Model = PointTransformerV3Model
    sys.modules["models.pointtransformer_v3"] = ptv3
    spc = types.ModuleType("models.spconv")
    spc.SparseConvModel = object
    sys.modules["models.spconv"] = spc


def main():
    rec = {}
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))  # repo root (for oracle)
    install_stubs(rec)
    sys.path.insert(0, REF)
    orig_tensor = torch.tensor

    def tensor_cpu(*a, **k):  # gs_utils.py:35 hard-codes device='cuda'
        if k.get("device") == "cuda":
            k["device"] = "cpu"
        return orig_tensor(*a, **k)

    torch.tensor = tensor_cpu
    import importlib
    gs_utils = importlib.import_module("utils.gs_utils")
    import models  # noqa: F401  (namespace package of the reference)
    fp_mod = importlib.import_module("models.feature_predictor")
    from splatformer_amd.scenes import make_cameras, make_scene

    # ---- 1. render glue, SH degree 1 and 0 -----------------------------------
    out = {}
    for deg in (1, 0, 3):
        s = make_scene(96, sh_degree=deg, seed=11 + deg)
        s["quats"][5] = float("nan")   # exercise the NaN-quaternion patch (gs_utils.py:47-51)
        cams = make_cameras(64, 48, n_views=2)
        cams["background_color"] = orig_tensor([0.1, 0.2, 0.3])
        c2w = cams["camera_to_worlds"][1]
        rec.clear()
        gs_utils.rasterize_gaussians_to_singleimg(
            s, c2w, orig_tensor(cams["cx"]), orig_tensor(cams["cy"]), orig_tensor(cams["fx"]),
            orig_tensor(cams["fy"]), orig_tensor(cams["width"]), orig_tensor(cams["height"]),
            cams["background_color"])
        p = f"deg{deg}_"
        for k, v in s.items():
            out[p + "in_" + k] = v.numpy()
        out[p + "c2w"] = c2w.numpy()
        out[p + "intr"] = np.array([cams["fx"], cams["fy"], cams["cx"], cams["cy"], cams["width"], cams["height"]],
                                   dtype=np.float64)
        out[p + "background"] = cams["background_color"].numpy()
        pr = rec["project"]
        out[p + "viewmat"] = pr["viewmat"].numpy()
        out[p + "scales"] = pr["scales"].numpy()
        out[p + "quats"] = pr["quats"].numpy()
        out[p + "proj_scalars"] = np.array([pr["glob_scale"], pr["fx"], pr["fy"], pr["cx"], pr["cy"],
                                            pr["img_height"], pr["img_width"], pr["block_width"]], dtype=np.float64)
        out[p + "opacity"] = rec["raster"]["opacity"].numpy()
        out[p + "colors"] = rec["raster"]["colors"].numpy()
        if "sh" in rec:
            out[p + "sh_deg"] = np.array(rec["sh"]["deg"])
            out[p + "sh_viewdirs"] = rec["sh"]["viewdirs"].numpy()
            out[p + "sh_coeffs"] = rec["sh"]["coeffs"].numpy()
    np.savez_compressed(os.path.join(OUT, "render_glue.npz"), **out)

    # ---- 2. FeaturePredictor (ptv3_base.gin head configuration) --------------
    torch.manual_seed(0)
    model = fp_mod.FeaturePredictor(
        backbone_type="PT", sh_degree=1,
        input_features=["means", "scales", "opacities", "quats", "features_dc", "features_rest"],
        input_feat_to_mlp=True,
        output_features=["means", "scales", "opacities", "quats", "features_dc", "features_rest"],
        output_head_nlayer=4, output_head_type="mlp-relu", output_head_width=128, output_features_type="res",
        res_feature_activation={"means": torch.nn.Tanh(), "features_dc": torch.nn.Identity(),
                                "features_rest": torch.nn.Identity(), "scales": torch.nn.Identity(),
                                "opacities": torch.nn.Identity(), "quats": torch.nn.Identity()},
        max_scale_normalized=1e-2, grid_resolution=384, resume_ckpt=None, input_embed_to_mlp=False,
        zeroinit=False, additional_info={"tome": "base", "r": 0.0})
    model.eval()
    s = make_scene(200, sh_degree=1, seed=5)
    rec.clear()
    with torch.no_grad():
        outs = model([s], [0])
    fo = {}
    for k, v in s.items():
        fo["in_" + k] = v.numpy()
    bi = rec["backbone_in"]
    fo["bb_coord"] = bi["coord"].numpy()
    fo["bb_grid_coord"] = bi["grid_coord"].numpy()
    fo["bb_offset"] = bi["offset"].numpy()
    fo["bb_feat"] = bi["feat"].numpy()
    fo["bb_grid_size"] = bi["grid_size"].numpy()
    fo["bb_out"] = rec["backbone_out"].numpy()
    for k, v in model.features_outputhead.state_dict().items():
        fo["head." + k] = v.numpy()
    for k, v in outs[0].items():
        fo["out_" + k] = v.numpy()
    np.savez_compressed(os.path.join(OUT, "feature_predictor.npz"), **fo)
    torch.tensor = orig_tensor
    so = scene_io_golden(rec)
    mo = metrics_golden()
    eo = export_golden(rec, gs_utils)
    print("wrote", sorted(out)[:4], "...", len(out), "render arrays;", len(fo), "feature-predictor arrays;",
          len(so), "scene-io arrays;", len(mo), "metrics arrays;", len(eo), "export arrays")


def export_golden(rec, gs_utils):
    import tempfile
    from splatformer_amd.scenes import make_cameras, make_scene
    eo = {}
    with tempfile.TemporaryDirectory() as root:
        for deg in (1, 0):
            s = make_scene(50, sh_degree=deg, seed=31 + deg)
            if deg == 0:
                s["features_rest"] = torch.zeros(50, 0, 3)
            rec.pop("ply_elements", None)
            gs_utils.export_ply_forviewer(s, os.path.join(root, "pc", f"deg{deg}.ply"))
            for k, v in s.items():
                eo[f"deg{deg}_in_{k}"] = v.numpy()
            eo[f"deg{deg}_vertices"] = rec["ply_elements"]
        cams = make_cameras(80, 60, n_views=3)
        cams_t = {k: (torch.as_tensor(v) if not isinstance(v, torch.Tensor) else v) for k, v in cams.items()}
        cams_t["camera_to_worlds"] = cams_t["camera_to_worlds"][:, :3, :4].contiguous()  # nerfstudio [V,3,4]
        gs_utils.prepare_viewer(cams_t, root, 1)
        eo["cam_c2w"] = cams_t["camera_to_worlds"].numpy()
        eo["cam_intr"] = np.array([float(cams_t[k]) for k in ("fx", "fy", "width", "height")])
        eo["cameras_json"] = np.array(open(os.path.join(root, "cameras.json")).read())
        eo["cfg_args"] = np.array(open(os.path.join(root, "cfg_args")).read())
    np.savez_compressed(os.path.join(OUT, "export.npz"), **eo)
    return eo


def metrics_golden():
    import importlib
    metrics = importlib.import_module("utils.metrics")
    g = torch.Generator().manual_seed(21)
    mo = {}
    for i, (n, h, w) in enumerate([(2, 40, 36), (3, 23, 17)]):
        a = torch.rand(n, 3, h, w, generator=g)
        b = (a + 0.1 * torch.randn(n, 3, h, w, generator=g)).clamp(0, 1)
        mo[f"b{i}_img1"], mo[f"b{i}_img2"] = a.numpy(), b.numpy()
        mo[f"b{i}_ssim"] = metrics.ssim(a, b, window_size=11, size_average=False).numpy()
        mo[f"b{i}_psnr"] = metrics.psnr(a, b).numpy()
    np.savez_compressed(os.path.join(OUT, "metrics.npz"), **mo)
    return mo


def make_scene_dirs(root, n=1200, seed=3):
    """Synthetic nerfstudio + colmap folders (our own files) for the scene-loading goldens."""
    import pickle
    from PIL import Image
    g = torch.Generator().manual_seed(seed)
    ns = os.path.join(root, "scene0", "splatfacto")
    os.makedirs(os.path.join(ns, "nerfstudio_models"), exist_ok=True)
    means = torch.randn(n, 3, generator=g) * torch.tensor([2.0, 1.0, 0.5]) + torch.tensor([0.3, -1.0, 2.0])
    means[7] = torch.tensor([40.0, 0.0, 0.0])            # outliers
    means[8] = torch.tensor([0.0, -35.0, 0.0])
    params = {"means": means, "scales": torch.randn(n, 3, generator=g) - 4.0,
              "quats": torch.randn(n, 4, generator=g), "opacities": torch.randn(n, 1, generator=g),
              "features_dc": torch.randn(n, 3, generator=g), "features_rest": torch.randn(n, 3, 3, generator=g) * 0.1}
    params["means"][11, 1] = float("nan")                # NaN rows in three attributes
    params["features_rest"][12, 2, 0] = float("nan")
    params["quats"][13, 3] = float("nan")
    params["scales"][14, 0] = float("-inf")             # inf after the log-scale shift
    ck = {"_model.gauss_params." + k: v for k, v in params.items()}
    ck["step"] = 29999
    torch.save(ck, os.path.join(ns, "nerfstudio_models", "step-000029999.ckpt"))
    c2w = lambda m: torch.cat([torch.linalg.qr(torch.randn(m, 3, 3, generator=g))[0],
                               torch.randn(m, 3, 1, generator=g) * 3], 2)
    meta = {"train_camera_to_worlds": c2w(5), "test_camera_to_worlds": c2w(12),
            "fx": torch.tensor(711.1), "fy": torch.tensor(711.1), "cx": torch.tensor(400.0),
            "cy": torch.tensor(400.0), "width": torch.tensor(800), "height": torch.tensor(800)}
    with open(os.path.join(ns, "camera_for-3d-denoise.pkl"), "wb") as f:
        pickle.dump(meta, f)
    cm = os.path.join(root, "colmap", "scene0")
    os.makedirs(os.path.join(cm, "images"), exist_ok=True)
    names = [f"frame_{i:03d}.png" for i in range(5)]
    names += [f"elevation{e}_azimuth{a}.png" for e in (30, 70, 80, 90) for a in (0, 120, 240)]
    for nm in names:
        open(os.path.join(cm, "images", nm), "wb").close()
    rgba = (torch.rand(6, 5, 4, generator=g) * 255).to(torch.uint8).numpy()
    img = os.path.join(root, "rgba.png")
    Image.fromarray(rgba, "RGBA").save(img)
    return ns, cm, params, meta, img


def scene_io_golden(rec):
    import importlib
    import tempfile
    GS = importlib.import_module("dataset.GS")
    so = {}
    with tempfile.TemporaryDirectory() as root:
        ns, cm, params, meta, img = make_scene_dirs(root)
        for k, v in params.items():
            so["in_" + k] = v.numpy()
        for k, v in meta.items():
            so["in_meta_" + k] = v.numpy()
        so["in_rgba"] = np.array(__import__("PIL.Image", fromlist=["Image"]).open(img))
        feats = ["means", "scales", "opacities", "quats", "features_dc", "features_rest"]
        rec["gin"] = {"FeaturePredictor.input_features": feats, "training.pretrain_steps": 0}
        for nd in (0, 3):
            ds = GS.SplatfactoDataset.__new__(GS.SplatfactoDataset)
            ds.remove_outlier_ndevs, ds.max_gs_num, ds.train_or_test = nd, 1000, "test"
            ds.folders, ds.load_pose_src = [(ns, cm)], "nerfstudio"
            scene = ds.load_scene(0)
            p = f"nd{nd}_"
            for k, v in scene["gs_params"].items():
                so[p + k] = v.numpy()
            so[p + "test_c2w"] = scene["meta"]["test_camera_to_worlds"].numpy()
            so[p + "train_c2w"] = scene["meta"]["train_camera_to_worlds"].numpy()
            so[p + "test_names"] = np.array([os.path.basename(x) for x in scene["test_imgs_path"]])
            so[p + "train_names"] = np.array([os.path.basename(x) for x in scene["train_imgs_path"]])
        ds = GS.SplatfactoDataset.__new__(GS.SplatfactoDataset)
        bg = torch.tensor([0.25, 0.5, 1.0])
        so["rgba_bg"] = bg.numpy()
        so["rgba_out"] = ds.read_image(img, background=bg).numpy()
    np.savez_compressed(os.path.join(OUT, "scene_io.npz"), **so)
    return so


if __name__ == "__main__":
    main()
