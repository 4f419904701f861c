"""In-refine vs isolated GEMM launches: the same stage-3 linears (C = 256: qkv, fc1, fc2 of
the config-B refine) timed where the refine issues them and replayed alone on the same tensors.

  run:        python tools/gemm_context.py run <outdir>        (GPU box; rocprofv3 passes: kernel trace, then SQ /
                                                               GRBM counters, then TCC hit/miss)
  summarize:  python tools/gemm_context.py summarize <outdir>

The program: 2 warm-up refines; 2 refines in which every linear whose shape is one of SHAPES is bracketed by two
marker kernels (its in-refine launch); then per shape the first recorded call replayed REPS times back to back on
its own inputs, bracketed by two markers.  labels.json (written by the program) names the brackets in order.
Per shape and context: median kernel duration (trace pass), effective clock = GRBM_GUI_ACTIVE / 8 XCDs /
duration (MI355X_MICROARCH.md, DVFS give-back), matrix-pipe busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
GRBM_GUI_ACTIVE / 8), wait share = SQ_WAIT_ANY / SQ_WAVE_CYCLES, L2 hit rate = TCC_HIT / (TCC_HIT + TCC_MISS).
"""
import csv
import glob
import os
import statistics
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SHAPES = {(37759, 768, 256): "qkv", (37759, 1024, 256): "fc1", (37759, 256, 1024): "fc2"}
REPS = 10
PASSES = {
    "trace": ["--kernel-trace"],
    "sq": ["--pmc", "GRBM_GUI_ACTIVE", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_VALU_MFMA_BUSY_CYCLES"],
    "tcc": ["--pmc", "TCC_HIT_sum", "TCC_MISS_sum", "GRBM_GUI_ACTIVE"],
}


def program():
    import json
    import torch
    from splatformer_amd import _lib
    from splatformer_amd import ptv3_ops as ops
    from splatformer_amd.feature_predictor import FeaturePredictor
    from splatformer_amd.scenes import make_scene, to_device
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = FeaturePredictor(sh_degree=1, zeroinit=False).eval().to(dev)
    scene = to_device(make_scene(100_000, sh_degree=1, seed=0), dev)
    for _ in range(2):
        model.refine_packed(scene)
    torch.cuda.synchronize()
    rec, labels = [], []
    orig = ops.linear
    mark = lambda: _lib.call("sfx_profile_marker", 0, _lib.stream())

    def linear(x, weight, bias=None, **kw):
        M = x.shape[0] if kw.get("rows") is None else kw["rows"]
        key = (M, weight.shape[0], weight.shape[1])
        if key not in SHAPES or kw.get("gather_idx") is not None:
            return orig(x, weight, bias, **kw)
        mark()  # each recorded launch bracketed by two markers
        out = orig(x, weight, bias, **kw)
        mark()
        labels.append(("refine", SHAPES[key]))
        if len(rec) < 64:
            rec.append((SHAPES[key], x, weight, bias, dict(kw)))
        return out

    ops.linear = linear
    for _ in range(2):
        model.refine_packed(scene)
    ops.linear = orig
    seen = set()
    for name, x, w, b, kw in rec:
        if name in seen:
            continue
        seen.add(name)
        kw = {k: v for k, v in kw.items() if k not in ("out", "y_amax")}
        mark()
        for _ in range(REPS):
            orig(x, w, b, **kw)
        mark()
        labels.append(("isolated", name))
    torch.cuda.synchronize()
    with open(os.environ["GEMM_CTX_LABELS"], "w") as f:
        json.dump(labels, f)
    print("recorded", sorted(seen), len(labels), flush=True)


def run(outdir):
    os.makedirs(outdir, exist_ok=True)
    for tag, opts in PASSES.items():
        os.environ["GEMM_CTX_LABELS"] = os.path.join(outdir, "labels.json")
        cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", *opts, "-d", os.path.join(outdir, tag), "-o", "run",
               "--output-format", "csv", "--", sys.executable, os.path.abspath(__file__), "program"]
        print("==", tag, flush=True)
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
        if r.returncode != 0:
            print(r.stdout.decode(errors="replace")[-2000:])
            sys.exit(r.returncode)


def summarize(outdir):
    import json
    labels = json.load(open(os.path.join(outdir, "labels.json")))

    def launches(tag):
        """label index -> dispatch ids of the GEMM launches between its two markers (dispatch order)."""
        f = glob.glob(os.path.join(outdir, tag, "**", "*kernel_trace.csv" if tag == "trace" else "*counter_collection.csv"),
                      recursive=True)[0]
        seen, rows = set(), []
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            if d not in seen:
                seen.add(d)
                rows.append((d, r["Kernel_Name"]))
        rows.sort()
        marks = [i for i, (d, k) in enumerate(rows) if "profile_marker_kernel" in k]
        assert len(marks) == 2 * len(labels), (tag, len(marks), len(labels))
        return [[rows[j][0] for j in range(marks[2 * i] + 1, marks[2 * i + 1]) if "gemm_kernel" in rows[j][1]]
                for i in range(len(labels))]

    tr = glob.glob(os.path.join(outdir, "trace", "**", "*kernel_trace.csv"), recursive=True)[0]
    dur = {int(r["Dispatch_Id"]): (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
           for r in csv.DictReader(open(tr))}
    cnt, ids = {}, {"trace": launches("trace")}
    for tag in ("sq", "tcc"):
        f = glob.glob(os.path.join(outdir, tag, "**", "*counter_collection.csv"), recursive=True)[0]
        c = defaultdict(dict)
        for r in csv.DictReader(open(f)):
            c[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        cnt[tag] = c
        ids[tag] = launches(tag)
    print(f"{'shape':>6s} {'ctx':>8s} {'n':>3s} {'us':>8s} {'GHz':>6s} {'MFMA%':>6s} {'wait%':>6s} {'L2hit%':>7s}")
    for name in ("qkv", "fc1", "fc2"):
        for ctx in ("refine", "isolated"):
            sel = [i for i, (c, nm) in enumerate(labels) if c == ctx and nm == name]
            if not sel:
                continue
            us = statistics.median(dur[d] for i in sel for d in ids["trace"][i])
            med = lambda tag, k, dflt=0.0: statistics.median(cnt[tag][d].get(k, dflt) for i in sel for d in ids[tag][i])
            ga, busy = med("sq", "GRBM_GUI_ACTIVE"), med("sq", "SQ_VALU_MFMA_BUSY_CYCLES")
            wa, wc = med("sq", "SQ_WAIT_ANY"), med("sq", "SQ_WAVE_CYCLES", 1.0)
            hit, miss = med("tcc", "TCC_HIT_sum"), med("tcc", "TCC_MISS_sum")
            n = sum(len(ids["trace"][i]) for i in sel)
            # the pmc passes serialise dispatches: their GRBM cycles over the trace pass's duration give the clock
            # the kernel ran at only approximately (profiled passes clock 2-5 % lower, DVFS give-back item 2)
            ghz = ga / 8 / (us * 1e3) if us > 0 else 0.0
            mfma = busy / (1024 * ga / 8) if ga > 0 else 0.0
            print(f"{name:>6s} {ctx:>8s} {n:3d} {us:8.1f} {ghz:6.2f} {100 * mfma:6.1f} {100 * wa / wc:6.1f} "
                  f"{100 * hit / max(1.0, hit + miss):7.1f}")


if __name__ == "__main__":
    if sys.argv[1] == "program":
        program()
    elif sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        summarize(sys.argv[2])
