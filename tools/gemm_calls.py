"""Per-call GEMM breakdown of one refine (config B workload, or --config E / A): every GEMM-family launch timed
in context (bench.GemmTimer: HIP events around each launch, real launch sequence), aggregated by
(op, M, N, K): calls, ms per scene, TFLOP/s.  GPU only: python tools/gemm_calls.py [--config B]"""
import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="B")
    ap.add_argument("--passes", type=int, default=3)
    a = ap.parse_args()
    n, _, _, sh, _ = bench.DEFAULTS[a.config]
    dev = torch.device("cuda")
    torch.manual_seed(0)
    bk = bench.DEPTH1 if a.config == "A" else {}
    model = FeaturePredictor(sh_degree=sh, zeroinit=False, backbone_kwargs=bk).eval().to(dev)
    scene = to_device(make_scene(n, sh_degree=sh, seed=0), dev)
    model.refine_packed(scene)
    runs = []
    for _ in range(a.passes):
        torch.cuda.synchronize()
        with bench.GemmTimer() as t:
            model.refine_packed(scene)
        runs.append(t.summary())
    runs.sort(key=lambda r: sum(p[0] for p in r))
    per = runs[len(runs) // 2]
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for ms, kind, shape, fl, by in per:
        k = agg[(kind,) + tuple(shape)]
        k[0] += 1
        k[1] += ms
        k[2] += fl
    tot = sum(v[1] for v in agg.values())
    for k, (c, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        dims = tuple(k[1:]) + (0,) * (3 - len(k[1:]))  # cpe_residual_ln (pair sums) has (rows, C)
        print(f"{k[0]:15s} M={dims[0]:6d} N={dims[1]:5d} K={dims[2]:5d} calls={c:3d} {ms:7.3f} ms "
              f"{fl / ms / 1e9:6.1f} TF/s")
    fl = sum(p[3] for p in per)
    print(f"total {tot:.2f} ms / scene, {fl / tot / 1e9:.1f} TF/s")


if __name__ == "__main__":
    main()
