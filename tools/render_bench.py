"""Eval-render timing on the bench workloads (config B: 100k SH1 9 x 800x800; E: 500k SH3 9 x 1920x1080):
the refined Gaussians of bench.py's model/scene, rendered with and without exact contribution culling
(SFX_RENDER_CULL), per-kernel times from torch.profiler-free HIP events around the whole render plus
intersection counts.  usage: python tools/render_bench.py [B|E] [reps]"""
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from splatformer_amd import _lib, gs_render  # noqa: E402
from splatformer_amd.feature_predictor import FeaturePredictor  # noqa: E402
from splatformer_amd.scenes import make_cameras, make_scene, to_device  # noqa: E402

CFG = {"B": (100_000, 800, 800, 1), "E": (500_000, 1920, 1080, 3)}


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "B"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    n, W, H, sh = CFG[cfg]
    dev = torch.device("cuda", 0)
    _lib.load()
    torch.manual_seed(0)
    model = FeaturePredictor(sh_degree=sh, zeroinit=False).eval().to(dev)
    scene = to_device(make_scene(n, sh_degree=sh, seed=0), dev)
    cams = to_device(make_cameras(W, H, n_views=9), dev)
    with torch.no_grad():
        out = model([scene], [0])[0]
    for name, gs in (("refined", out), ("input", scene)):
        for cull in (False, True, False, True):
            gs_render.RENDER_CULL = cull
            with torch.no_grad():
                r, a, m = gs_render.render_views_meta(gs, cams)
                ts = []
                for _ in range(reps):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    gs_render.rasterize_gaussians_to_multiimgs(gs, cams)
                    torch.cuda.synchronize()
                    ts.append(1e3 * (time.perf_counter() - t0))
            ni = m["isect_sorted"].numel() if "isect_sorted" in m else 0
            print(f"{cfg} {name:8s} cull={int(cull)} isect={ni:9d} render 9 views median {statistics.median(ts):7.3f} ms "
                  f"(min {min(ts):7.3f})", flush=True)


def train_main(reps=5):
    """Training render (autograd glue, gs_utils.py:32-113) of the bench scene's 4 training views at 800x800:
    forward + backward per view, cull on / off; per-kernel times come from a rocprofv3 kernel trace."""
    n, W, H, sh = CFG["B"]
    dev = torch.device("cuda", 0)
    _lib.load()
    from splatformer_amd import gsplat_compat
    scene = to_device(make_scene(n, sh_degree=sh, seed=0), dev)
    cams = to_device(make_cameras(W, H, n_views=4), dev)
    params = {k: v.clone().requires_grad_(True) for k, v in scene.items()}
    for cull in (False, True, False, True):
        gsplat_compat.CULL = cull
        ts = []
        for it in range(reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rgbs, _ = gs_render.rasterize_gaussians_to_multiimgs(params, cams)
            loss = sum(r.sum() for r in rgbs)
            loss.backward()
            torch.cuda.synchronize()
            if it:
                ts.append(1e3 * (time.perf_counter() - t0))
        g = params["means"].grad.norm().item()
        for p in params.values():
            p.grad = None
        print(f"train render 4 views fwd+bwd cull={int(cull)} median {statistics.median(ts):7.3f} ms "
              f"(min {min(ts):7.3f}) |grad means| {g:.6e}", flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "train":
    train_main()
    sys.exit(0)


if __name__ == "__main__":
    main()
