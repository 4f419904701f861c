"""Timing ablations of the GEMM family on the config-B refine launches (which part bounds gemm_kernel?).
Each distinct launch of one refine pass is timed with the default tile choice; run once per SFX_GEMM_DEBUG value
(bit 0 no MFMAs, 1 no operand loads, 2 no epilogue, 3 no LDS staging -- results wrong, timing only):
    SFX_GEMM_DEBUG=<bits> python tools/gemm_ablate.py [n_gaussians] > out.jsonl       (GPU only)"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from gemm_tune import GemmRecorder, timeit  # noqa: E402
from splatformer_amd.feature_predictor import FeaturePredictor  # noqa: E402
from splatformer_amd.scenes import make_scene, to_device  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = FeaturePredictor(sh_degree=1, zeroinit=False).eval().to(dev)
    scene = to_device(make_scene(n, sh_degree=1, seed=0), dev)
    model.refine_packed(scene)
    with GemmRecorder() as rec:
        model.refine_packed(scene)
    torch.cuda.synchronize()
    mode = int(os.environ.get("SFX_GEMM_DEBUG", "0"))
    seen = {}
    for kind, fl, fn, shape in rec.calls:
        key = (kind,) + tuple(shape)
        if key in seen:
            seen[key][0] += 1
            continue
        seen[key] = [1, timeit(fn, reps=20)]
    for key, (cnt, us) in seen.items():
        print(json.dumps({"mode": mode, "key": key, "calls": cnt, "us": round(us, 2)}), flush=True)
    print(json.dumps({"mode": mode, "total_us": round(sum(c * u for c, u in seen.values()), 1)}), flush=True)


if __name__ == "__main__":
    main()
