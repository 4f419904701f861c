"""Which Python call sites launch the torch-side copies / fills of one config-B step (GPU only).

torch.profiler over one refine + 9-view render; every aten copy/fill/zero op is attributed to its innermost
splatformer_amd frame and aggregated: calls and device time per (op, file:line).
python tools/torch_ops_prof.py"""
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from splatformer_amd import _lib  # noqa: E402
from splatformer_amd.feature_predictor import FeaturePredictor  # noqa: E402
from splatformer_amd.gs_render import rasterize_gaussians_to_multiimgs  # noqa: E402
from splatformer_amd.scenes import make_cameras, make_scene, to_device  # noqa: E402


def main():
    dev = torch.device("cuda")
    _lib.load()
    torch.manual_seed(0)
    cams = to_device(make_cameras(800, 800, n_views=9), dev)
    model = FeaturePredictor(sh_degree=1, zeroinit=False).eval().to(dev)
    scene = to_device(make_scene(100000, sh_degree=1, seed=0), dev)

    def step():
        out = model([scene], [0])[0]
        return rasterize_gaussians_to_multiimgs(out, cams)

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    agg = collections.defaultdict(lambda: [0, 0.0])
    for ev in prof.events():
        name = ev.name
        if not any(k in name for k in ("copy_", "fill_", "zero_", "aten::zeros", "aten::empty_like", "index", "cat",
                                       "aten::to", "clone", "contiguous")):
            continue
        if ev.device_type != torch.autograd.DeviceType.CPU:
            continue
        site = "?"
        for fr in (ev.stack or []):
            if "splatformer_amd" in fr or "bench" in fr:
                site = fr.split("/")[-1]
                break
        t = float(getattr(ev, "device_time_total", 0.0) or 0.0)
        a = agg[(name, site)]
        a[0] += 1
        a[1] += t
    for (name, site), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:60]:
        print(f"{c:4d} {t:9.1f} us  {name:28s} {site}")


if __name__ == "__main__":
    main()
