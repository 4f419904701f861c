"""Per-kernel-family evidence for the config-B step: HBM bytes (rocprofv3 FETCH_SIZE x 2 +
WRITE_SIZE, MI355X_MICROARCH.md: gfx950 FETCH_SIZE counts half the bytes of wide reads), achieved GB/s against the
8 TB/s HBM peak, durations, and the matrix-pipe utilisation of the MFMA kernels (SQ_VALU_MFMA_BUSY_CYCLES over the
SIMD-cycles of the dispatch) -- steady-state units only: `bench.py --profile-only --markers` brackets every timed
step with a marker kernel, and each figure is per unit (one refine + 9 renders), median over the marked units.

Run on the GPU box (each counter group is its own rocprofv3 pass, as the guide prescribes):
  python tools/kernel_pmc.py run <outdir> [bench args...]      -> CSVs under <outdir>
  python tools/kernel_pmc.py summarize <outdir> > summary.txt
"""
import csv
import glob
import os
import re
import statistics
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = {
    "trace": ["--kernel-trace"],
    "fetch": ["--pmc", "FETCH_SIZE"],
    "write": ["--pmc", "WRITE_SIZE"],
    "sq": ["--pmc", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_MFMA", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
           "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "GRBM_GUI_ACTIVE"],
    "sq2": ["--pmc", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_WAIT_INST_LDS", "SQ_BUSY_CYCLES",
            "GRBM_GUI_ACTIVE"],
}
FAMILIES = [  # (family, kernel-name regex) -- first match wins
    ("gemm", r"^gemm_kernel|^wgrad_kernel"),
    ("mlp (fused Block MLP)", r"^mlp_kernel"),
    ("subm pair-sum LayerNorm", r"^cpe_residual_ln4_kernel<\d+, \d+, true>"),
    ("fused subm conv + CPE LN", r"^subm_cpe_ln_kernel"),
    ("fused output heads", r"^heads_kernel"),
    ("pair-sum LN + qkv (fused)", r"^cpe_ln_qkv_kernel"),
    ("point embedding", r"^point_embed"),
    ("attention", r"^window_attn"),
    ("attention + proj (fused)", r"^attn_proj_kernel"),
    ("rasterizer", r"^rasterize_fwd"),
    ("render prep/project + records", r"^render_prep_project|^pack_raster_records|^isect_emit|^tile_bins"),
    ("radix sort + scans", r"^radix_|^scan_"),
    ("serialization", r"^serialize_"),
    ("subm maps", r"^subm_(?!cpe)"),
    ("pooling", r"^pool_|^segment_"),
    ("layernorm", r"^layernorm|^cpe_residual_ln"),
    ("copies/fills", r"^__amd_rocclr"),
]
CUS, SIMDS = 256, 1024
HBM_PEAK = 8000.0  # GB/s
MFMA_CYCLES = {"f16_32x32x16": 32}


def short(name):
    m = re.search(r"(\w+)(<[^()]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else name


def family(name):
    s = short(name)
    for fam, rx in FAMILIES:
        if re.search(rx, s):
            return fam
    return "other"


def run(outdir, bench_args):
    os.makedirs(outdir, exist_ok=True)
    argv = [sys.executable, os.path.join(ROOT, "bench.py"), "--profile-only", "--markers", "--steps", "3",
            "--warmup", "2", *bench_args]
    for tag, opts in PASSES.items():
        cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", *opts, "-d", os.path.join(outdir, tag), "-o", "run",
               "--output-format", "csv", "--", *argv]
        print("==", tag, flush=True)
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
        if r.returncode != 0:
            print(r.stdout.decode(errors="replace")[-2000:])
            sys.exit(r.returncode)


def _units(rows):
    """rows: (dispatch_id, kernel_name, value) -> list of per-unit {family: [values]} between markers."""
    rows.sort()
    marks = [d for d, k, _ in rows if "profile_marker_kernel" in k]
    units = []
    for a, b in zip(marks[:-1], marks[1:]):
        u = defaultdict(list)
        for d, k, v in rows:
            if a < d < b:
                u[(family(k), short(k))].append(v)
        units.append(u)
    return units


def load_counters(path):
    per = defaultdict(list)  # counter -> rows
    with open(path) as f:
        for r in csv.DictReader(f):
            per[r["Counter_Name"]].append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    return per


def load_trace(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))))
    return rows


def per_unit_sum(units, key_fn):
    """median over units of the sum of the values selected by key_fn(key) -> bool."""
    return statistics.median([sum(sum(v) for k, v in u.items() if key_fn(k)) for u in units]) if units else 0.0


def summarize(outdir):
    f = lambda tag, pat: glob.glob(os.path.join(outdir, tag, "**", pat), recursive=True)[0]
    trace = _units(load_trace(f("trace", "*kernel_trace.csv")))
    fetch = _units(load_counters(f("fetch", "*counter_collection.csv"))["FETCH_SIZE"])
    write = _units(load_counters(f("write", "*counter_collection.csv"))["WRITE_SIZE"])
    sq = load_counters(f("sq", "*counter_collection.csv"))
    sq2 = load_counters(f("sq2", "*counter_collection.csv"))
    sqc = {c: _units(v) for c, v in sq.items()}
    sqc.update({c + "#2": _units(v) for c, v in sq2.items()})
    fams = sorted({k[0] for u in trace for k in u})
    tot_ms = per_unit_sum(trace, lambda k: True) / 1e6
    print(f"# per unit (1 refine + 9 views of config B), median of {len(trace)} marked units; kernel time sum "
          f"{tot_ms:.3f} ms")
    print(f"{'family':32s} {'ms':>7s} {'launch':>6s} {'HBM MB':>9s} {'GB/s':>7s} {'%8TB/s':>7s} {'MFMA%':>6s} "
          f"{'wait%':>6s}")
    rows = []
    for fam in fams:
        sel = lambda k, fam=fam: k[0] == fam
        ms = per_unit_sum(trace, sel) / 1e6
        n = statistics.median([sum(len(v) for k, v in u.items() if sel(k)) for u in trace])
        hbm = (2 * per_unit_sum(fetch, sel) + per_unit_sum(write, sel)) * 1024.0
        gbs = hbm / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        busy = per_unit_sum(sqc.get("SQ_VALU_MFMA_BUSY_CYCLES", []), sel)
        grbm = per_unit_sum(sqc.get("GRBM_GUI_ACTIVE", []), sel)  # summed over the 8 XCDs
        mfma = busy / (SIMDS * grbm / 8) if grbm > 0 else 0.0
        wc = per_unit_sum(sqc.get("SQ_WAVE_CYCLES", []), sel)
        wa = per_unit_sum(sqc.get("SQ_WAIT_ANY", []), sel)
        rows.append((ms, fam, n, hbm, gbs, mfma, wa / wc if wc else 0.0))
    for ms, fam, n, hbm, gbs, mfma, wait in sorted(rows, reverse=True):
        print(f"{fam:32s} {ms:7.3f} {n:6.0f} {hbm / 1e6:9.1f} {gbs:7.0f} {100 * gbs / HBM_PEAK:6.1f}% "
              f"{100 * mfma:5.1f}% {100 * wait:5.1f}%")
    print("\n# per kernel (top 30 by time)")
    keys = sorted({k for u in trace for k in u}, key=lambda k: -per_unit_sum(trace, lambda kk, k=k: kk == k))
    for k in keys[:30]:
        sel = lambda kk, k=k: kk == k
        ms = per_unit_sum(trace, sel) / 1e6
        hbm = (2 * per_unit_sum(fetch, sel) + per_unit_sum(write, sel)) * 1024.0
        busy = per_unit_sum(sqc.get("SQ_VALU_MFMA_BUSY_CYCLES", []), sel)
        grbm = per_unit_sum(sqc.get("GRBM_GUI_ACTIVE", []), sel)
        conf = per_unit_sum(sqc.get("SQ_LDS_BANK_CONFLICT#2", []), sel)
        lds = per_unit_sum(sqc.get("SQ_LDS_IDX_ACTIVE#2", []), sel)
        print(f"{k[1][:60]:60s} {ms:7.3f} ms {hbm / 1e6:9.1f} MB {hbm / max(ms, 1e-9) / 1e6:7.0f} GB/s "
              f"MFMA {100 * busy / (SIMDS * grbm / 8) if grbm else 0:5.1f}% LDS-conflict "
              f"{100 * conf / lds if lds else 0:5.1f}%")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], sys.argv[3:])
    else:
        summarize(sys.argv[2])
