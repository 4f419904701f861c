"""Measure every (tile configuration, Stream-K) for each distinct GEMM launch of one refine pass (config B
workload) and print the fastest -- the data behind gemm.hip's tuned table.  GPU only:
python tools/gemm_tune.py [n_gaussians] [kind filter, e.g. subm_conv, or all] [sh_degree] > table.txt"""
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


class GemmRecorder:
    """Records the GEMM launches (ptv3_ops.linear / subm_conv / grouped_linear) of one refine pass as
    re-runnable closures writing into scratch outputs."""

    def __enter__(self):
        self.calls = []
        self._lin, self._conv, self._grp = ops.linear, ops.subm_conv, ops.grouped_linear
        rec = self

        def lin(x, weight, bias=None, **kw):
            res = rec._lin(x, weight, bias, **kw)
            out = res[0] if isinstance(res, tuple) else res
            M, (N, K) = out.shape[0], weight.shape
            kw2 = dict(kw, out=torch.empty_like(out))
            if kw.get("pre_out") is not None:
                kw2["pre_out"] = torch.empty_like(kw["pre_out"])
            rec.calls.append(("linear", 2.0 * M * N * K, lambda: rec._lin(x, weight, bias, **kw2), (M, N, K)))
            return res

        def conv(x, smap, weight, bias, out=None, **kw):
            o = rec._conv(x, smap, weight, bias, out=out, **kw)
            n, cin = x.shape
            cout = weight.shape[0]
            scratch = torch.empty(n, cout, device=x.device, dtype=torch.float32)
            npairs = smap.lists(True).num_pairs if smap.centre_pref else n + smap.num_pairs
            rec.calls.append(("subm_conv", 2.0 * npairs * cin * cout,
                              lambda: rec._conv(x, smap, weight, bias, out=scratch, **kw), (n, cout, cin)))
            return o

        def grp(x, weight, bias, groups, **kw):
            res = rec._grp(x, weight, bias, groups, **kw)
            out = res[0] if isinstance(res, tuple) else res
            G, N, K = weight.shape
            scratch = torch.empty_like(out)
            rec.calls.append(("grouped_linear", 2.0 * x.shape[0] * G * N * K,
                              lambda: rec._grp(x, weight, bias, groups, **dict(kw, out=scratch)), (x.shape[0], G * N, K)))
            return res

        ops.linear, ops.subm_conv, ops.grouped_linear = lin, conv, grp
        return self

    def __exit__(self, *a):
        ops.linear, ops.subm_conv, ops.grouped_linear = self._lin, self._conv, self._grp


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
    only = sys.argv[2] if len(sys.argv) > 2 and sys.argv[2] != "all" else None
    sh = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = FeaturePredictor(sh_degree=sh, zeroinit=False).eval().to(dev)
    scene = to_device(make_scene(n, sh_degree=sh, seed=0), dev)
    model.refine_packed(scene)
    with GemmRecorder() as rec:
        model.refine_packed(scene)
    torch.cuda.synchronize()
    seen = {}
    for kind, fl, fn, shape in rec.calls:
        key = (kind,) + tuple(shape)
        if only and kind != only:
            continue
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
