"""Host-side (Python) cost of the config-B step: cProfile over timed steps, top functions by own time, plus the
wall time per step.  When the step's host enqueue time approaches its GPU time, the GPU idles between launches
(tools/gpu_gaps.sh shows it as a median gap of several us).  usage: python tools/host_profile.py [steps]"""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from splatformer_amd import _lib  # noqa: E402
from splatformer_amd.feature_predictor import FeaturePredictor  # noqa: E402
from splatformer_amd.gs_render import rasterize_gaussians_to_multiimgs  # noqa: E402
from splatformer_amd.scenes import make_cameras, make_scene, to_device  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    _lib.load()
    torch.manual_seed(0)
    model = FeaturePredictor(sh_degree=1, zeroinit=False).eval().to(dev)
    scene = to_device(make_scene(100_000, sh_degree=1, seed=0), dev)
    cams = to_device(make_cameras(800, 800, n_views=9), dev)

    def step():
        out = model([scene], [0])[0]
        return rasterize_gaussians_to_multiimgs(out, cams)[0]

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    print(f"wall {1e3 * (time.perf_counter() - t0) / steps:.3f} ms/step (no profiler)")
    # host-only cost without the profiler's per-call overhead: wall time minus the time spent blocked in event
    # waits (the library's host reads: HostRead.get -> Event.synchronize) -- what the Python side itself costs
    waited = [0.0]
    orig_sync = torch.cuda.Event.synchronize

    def timed_sync(ev):
        a = time.perf_counter()
        orig_sync(ev)
        waited[0] += time.perf_counter() - a
    torch.cuda.Event.synchronize = timed_sync
    try:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        t_enq = time.perf_counter()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
    finally:
        torch.cuda.Event.synchronize = orig_sync
    print(f"host python {1e3 * (t_enq - t0 - waited[0]) / steps:.3f} ms/step (wall to last enqueue "
          f"{1e3 * (t_enq - t0) / steps:.3f} ms, blocked in host reads {1e3 * waited[0] / steps:.3f} ms, "
          f"GPU tail after the last enqueue {1e3 * (t1 - t_enq):.3f} ms)")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(45)
    st.sort_stats("cumtime").print_stats(30)


if __name__ == "__main__":
    main()
