"""Per-call GEMM breakdown of one refine pass of the bench workload (config B), aggregated by
(op, M, N, K): calls, ms per scene, TFLOP/s.  GPU only: python tools/gemm_calls.py"""
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from splatformer_amd.feature_predictor import FeaturePredictor  # noqa: E402
from splatformer_amd.scenes import make_scene, to_device  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = FeaturePredictor(sh_degree=1, zeroinit=False).eval().to(dev)
    scene = to_device(make_scene(100_000, sh_degree=1, seed=0), dev)
    model.refine_packed(scene)
    with bench.GemmRecorder() as rec:
        model.refine_packed(scene)
    torch.cuda.synchronize()
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for kind, fl, fn, shape in rec.calls:
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        a = agg[(kind,) + tuple(shape)]
        a[0] += 1
        a[1] += ms
        a[2] += fl
    tot = sum(v[1] for v in agg.values())
    for k, (c, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k[0]:15s} M={k[1]:6d} N={k[2]:5d} K={k[3]:5d} calls={c:3d} {ms:7.3f} ms {fl / ms / 1e9:6.1f} TF/s")
    print(f"total {tot:.2f} ms / scene")


if __name__ == "__main__":
    main()
