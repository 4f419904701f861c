"""Measure every (tile configuration, Stream-K) for each distinct GEMM launch of one refine pass (config B
workload) and print the fastest -- the data behind gemm.hip's tuned table.  GPU only:
python tools/gemm_tune.py [n_gaussians] > table.txt"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from splatformer_amd import ptv3_ops as ops  # noqa: E402
from splatformer_amd.feature_predictor import FeaturePredictor  # noqa: E402
from splatformer_amd.scenes import make_scene, to_device  # noqa: E402


def timeit(fn, reps=8):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = FeaturePredictor(sh_degree=1, zeroinit=False).eval().to(dev)
    scene = to_device(make_scene(n, sh_degree=1, seed=0), dev)
    model.refine_packed(scene)
    with bench.GemmRecorder() as rec:
        model.refine_packed(scene)
    torch.cuda.synchronize()
    seen = {}
    for kind, fl, fn, shape in rec.calls:
        key = (kind,) + tuple(shape)
        if key in seen:
            seen[key][0] += 1
            continue
        res = {}
        for cfg in [-1] + list(range(ops.GEMM_NUM_CONFIGS)):
            for sk in (0, 1):
                ops.gemm_force_config(cfg, sk if cfg >= 0 else -1)
                if cfg < 0 and sk == 1:
                    continue
                res[f"{cfg}/{sk}"] = timeit(fn)
        ops.gemm_force_config(-1, -1)
        best = min(res, key=res.get)
        seen[key] = [1, res, best]
        print(json.dumps({"key": key, "model_us": round(res["-1/0"], 1), "best": best,
                          "best_us": round(res[best], 1), "all": {k: round(v, 1) for k, v in res.items()}}), flush=True)
    tot_m = sum(c * r["-1/0"] for c, r, b in seen.values())
    tot_b = sum(c * r[b] for c, r, b in seen.values())
    print(f"# per scene: cost model {tot_m / 1e3:.2f} ms, best {tot_b / 1e3:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
