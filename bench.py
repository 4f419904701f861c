"""Benchmark of the SplatFormer hot path on MI355X (BASELINE.json configs).

Default (the driver's line) = config B: refined renders/sec on 100k-Gaussian x 800x800 scenes.  One step =
one scene per rank: FeaturePredictor forward (full ptv3_base PTv3 + heads, fp32-accurate) over 100k
Gaussians, then the 9 OOD test views (800x800) of the refined Gaussians through the gsplat-v0.1.11-semantics
renderer -- the reference's evaluation() hot loop (train.py:86-100).  Synthetic seeded scene and random-init
weights of the ptv3_base architecture (no datasets/checkpoints offline).

Multi-GPU: one process per GPU.  `python bench.py --gpus N` (N > 1, outside torchrun) starts
`torch.distributed.run --nproc-per-node N` as a child process before anything touches the GPU and exits
with its status; under torchrun (WORLD_SIZE set) every rank refines and renders its own scene (weak scaling,
no collective on the data path; barrier + max-over-ranks timing only), `n_gpus` = the real world size.

--config A: 20k Gaussians SH0 (Cin 14), depth-1 PTv3, 4 views 256x256 (the reference's CPU-runnable case).
--config C: training -- a step = a batch of 8 scenes (100k GS, SH1), each refined in train mode, rendered to
  4 training views (800x800), image-L1 loss, backward through renderer + refiner, then clip + Adam
  (train.py:236-303); renders/s = 8*4 / step time.
--config D: DDP training -- per rank one scene per micro-step, 4 micro-steps per optimiser step (accumulate
  4), RCCL all-reduce of the gradient bucket + SyncBatchNorm; a step = one optimiser step.
--config E: 500k Gaussians, SH3, 1920x1080, 9 views, forward (HBM-bound stress).

Prints ONE JSON line (rank 0) with
  * `roofline` for the dominant kernel family (the fp32-accurate MFMA GEMMs): algorithmic FLOP of every GEMM
    launch of one unit of work (a refine; for C/D one training micro-step, forward + backward) / the summed
    in-context launch durations (HIP events around each launch on the launch stream, in the real sequence,
    median of 3 passes); `algorithmic_bytes` of the same launches; `traffic` = HBM bytes of those launches
    from rocprofv3 PMC passes run by this script (child processes; 2*FETCH_SIZE + WRITE_SIZE per
    MI355X_MICROARCH.md), or null when the profiler is unavailable;
  * `cpu_baseline`: the CPU oracle (oracle/) on the box's host cores, rank 0 at N=1 only (protocol below).
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import platform
import shutil
import socket
import statistics
import subprocess
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
F16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense fp16 / bf16 MFMA (no sparsity)
# The GEMM computes fp32-accurate products as three fp16 term products (fp16x2 split operands, gemm.hip): its
# fp32-equivalent ceiling is the dense fp16 peak / 3.
SPLIT_PEAK_TFLOPS = round(F16_MFMA_PEAK_TFLOPS / 3, 1)
HBM_PEAK_GBS = 8000.0
# kernel-name prefixes of the dominant family: the GEMMs, the fused Block MLP, the fused SubM conv + CPE
# LayerNorm (subm_fused.hip), the fused output heads (heads.hip) and, since round 6, the fused attention + output
# projection (attn_proj.hip: it absorbed the projection GEMMs)
GEMM_FAMILY = ("gemm_kernel", "wgrad_kernel", "mlp_kernel", "subm_cpe_ln_kernel", "heads_kernel", "attn_proj_kernel",
               "cpe_ln_qkv_kernel")


def in_family(kernel_name: str) -> bool:
    """GEMM-family dispatch: the GEMM kernels, and the LayerNorm kernel that sums SubM pair partials (the
    conv's own reduction when it stores per-pair rows: `cpe_residual_ln4_kernel<G, NV, true>`)."""
    return any(p in kernel_name for p in GEMM_FAMILY) or (
        "cpe_residual_ln4_kernel<" in kernel_name and ", true>" in kernel_name)

DEFAULTS = {  # n, res, views, sh, batch
    "A": (20_000, "256", 4, 0, 1), "B": (100_000, "800", 9, 1, 1), "C": (100_000, "800", 4, 1, 8),
    "D": (100_000, "800", 4, 1, 4), "E": (500_000, "1920x1080", 9, 3, 1)}
DEPTH1 = dict(enc_depths=(1, 1, 1, 1, 1), dec_depths=(1, 1, 1, 1))


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=sorted(DEFAULTS), default="B")
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--res", type=str, default=None, help="W or WxH")
    ap.add_argument("--views", type=int, default=None)
    ap.add_argument("--train-prec", choices=["fp32", "amp"], default="fp32",
                    help="configs C/D: refiner precision; amp = the reference's enable_amp (train.py:240) class")
    ap.add_argument("--sh", type=int, default=None)
    ap.add_argument("--batch", type=int, default=None, help="scenes per step (C) / micro-steps (D)")
    ap.add_argument("--flash", action="store_true",
                    help="PointTransformerV3Model.enable_flash=True (K=1024 windows, pointtransformer_v3.py:121-123)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-psnr", action="store_true", help="skip the PSNR delta vs the oracle (eval configs)")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC passes")
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="Gaussians in the CPU-oracle sample (default: the whole scene)")
    ap.add_argument("--profile-only", action="store_true", help="skip roofline probe, traffic and CPU baseline")
    ap.add_argument("--markers", action="store_true",
                    help="launch sfx_profile_marker before every timed step and after the last (PMC passes)")
    ap.add_argument("--gemm-calls", type=str, default=None,
                    help="write the roofline probe's per-launch list (kind, shape, ms, TF/s; median pass) to this file")
    ap.add_argument("--dry-launch", action="store_true", help=argparse.SUPPRESS)  # launcher test: no GPU work
    a = ap.parse_args(argv)
    dflt = DEFAULTS[a.config]
    a.n = a.n if a.n is not None else dflt[0]
    res = a.res if a.res is not None else dflt[1]
    a.width, a.height = (int(res.split("x")[0]), int(res.split("x")[1])) if "x" in res else (int(res), int(res))
    a.views = a.views if a.views is not None else dflt[2]
    a.sh = a.sh if a.sh is not None else dflt[3]
    a.batch = a.batch if a.batch is not None else dflt[4]
    return a


# ---- multi-GPU launcher ---------------------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_cmd(gpus: int, argv, port: int):
    """The torchrun command that runs this script once per GPU (one process per GPU, rendezvous on
    127.0.0.1); the children see WORLD_SIZE and do not relaunch."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def needs_launch(gpus: int, env=None) -> bool:
    env = os.environ if env is None else env
    return gpus > 1 and "WORLD_SIZE" not in env


def world_size_check(gpus: int, world: int) -> None:
    if gpus not in (1, world):  # --gpus 1 is the default: accept any torchrun world
        raise SystemExit(f"bench.py: --gpus {gpus} but the launcher started {world} ranks")


# ---- GEMM family: in-context launch timing, FLOP and byte accounting -----------------------------------------
def _gemm_cost(kind, args, kw, res):
    """(FLOP, algorithmic bytes, shape) of one GEMM-family launch (fp32 operands, 4-byte elements)."""
    f4 = 4
    if kind == "linear":
        x, w = args[0], args[1]
        out = res[0] if isinstance(res, tuple) else res
        M, (N, K) = out.shape[0], w.shape
        by = (M * K + N * K + M * N) * f4
        by += sum(M * N * f4 for k in ("residual", "pre_out") if kw.get(k) is not None)
        return 2.0 * M * N * K, by, (M, N, K)
    if kind == "grouped_linear":
        x, w = args[0], args[1]
        G, N, K = w.shape
        M = x.shape[0]
        return 2.0 * M * G * N * K, (M * G * K + G * N * K + M * G * N) * f4, (M, G * N, K)
    if kind == "subm_conv":
        x, smap, w = args[0], args[1], args[2]
        n, cin = x.shape
        cout = w.shape[0]
        fl = 2.0 * (n + smap.num_pairs) * cin * cout
        return fl, (n * cin + 27 * cin * cout + n * cout + 27 * n) * f4, (n, cout, cin)
    if kind == "linear_bwd_data":
        dy, wt = args[0], args[1]
        M, N = dy.shape
        K = wt.shape[0]
        by = (M * N + K * N + M * K) * f4 + (M * K * f4 if kw.get("dact_pre") is not None else 0)
        return 2.0 * M * N * K, by, (M, K, N)
    if kind == "linear_wgrad":
        dy, x = args[0], args[1]
        M, N = dy.shape
        K = x.shape[1]
        return 2.0 * M * N * K, (M * N + M * K + 2 * N * K) * f4, (N, K, M)
    if kind == "subm_conv_bwd_data":
        dy, smap, wt, dx = args[0], args[1], args[2], args[3]
        n, cout = dy.shape
        cin = dx.shape[1]
        fl = 2.0 * (n + smap.num_pairs) * cin * cout
        return fl, (n * cout + 27 * cin * cout + 2 * n * cin + 27 * n) * f4, (n, cin, cout)
    if kind == "block_mlp":  # fused LN2 + fc1 + GELU + fc2 + residual (csrc/mlp.hip): the two GEMMs' FLOPs
        x = args[0]
        M, C = x.shape
        return 16.0 * M * C * C, (2 * M * C + 8 * C * C + 12 * C) * f4, (M, 4 * C, C)
    if kind == "cpe_residual_ln":  # timed only with SubM pair partials: the conv's own pair summation
        return 0.0, 0, tuple(args[1].shape)
    if kind == "subm_cpe_ln":  # fused conv (every active (out, in) pair incl. the centre) + its LayerNorm tail
        xc, smap = args[0], args[2]
        n, C = xc.shape
        nbr = smap.nbr
        # pair count read after the pass (a host read here would stall the launch sequence being timed)
        fl = lambda: 2.0 * float((nbr >= 0).sum()) * C * C
        return fl, (27 * n + 3 * n * C + 2 * n * C + 27 * C * C) * f4, (n, C, C)
    if kind == "heads":  # 6 x (kin -> 128 -> 128 -> 128 -> c_f) MLPs + residual, one launch
        x, kin, out_dim = args[0], args[1], args[3]
        M = x.shape[0]
        ng = len(args[5]) - 1
        fl = 2.0 * M * (ng * (kin * 128 + 2 * 128 * 128) + 128 * out_dim)
        return fl, (M * x.shape[1] + M * out_dim + ng * (kin * 128 + 2 * 128 * 128) + out_dim * 128) * f4, \
            (M, ng * 128, kin)
    if kind == "cpe_ln_qkv":  # pair-sum LayerNorms + the qkv projection (its GEMM FLOPs), one launch
        x = args[1]
        M, C = x.shape
        return 6.0 * M * C * C, (3 * M * C + 3 * M * C + 3 * C * C) * f4, (M, 3 * C, C)
    if kind == "window_attention_proj":  # fused attention (QK^T + PV over K-key windows) + projection + residual
        qkv, K, C = args[0], args[4], args[6]
        n = qkv.shape[0]
        return n * (4.0 * K * C + 2.0 * C * C), (n * 3 * C + 2 * n * C + C * C + C) * f4, (n, C, K)
    raise KeyError(kind)


class GemmTimer:
    """Wraps the GEMM-family entry points (ptv3_ops.linear / subm_conv / grouped_linear, train_ops
    linear_bwd_data / linear_wgrad / subm_conv_bwd_data) for one pass of real work: HIP events recorded on the
    launch stream around each launch, in the real launch sequence (no replay, caches as they are).  A SubM conv
    that stores per-pair partial rows (ptv3_ops.SubmPartials) finishes in its consumer, cpe_residual_ln, which
    sums them: those launches are timed with the family too (0 FLOP), so the family's TF/s covers the whole
    conv."""

    def __init__(self):
        self.calls = []

    def __enter__(self):
        from splatformer_amd import ptv3_ops, train_ops
        self._saved = []
        for mod, name in [(ptv3_ops, "linear"), (ptv3_ops, "subm_conv"), (ptv3_ops, "grouped_linear"),
                          (train_ops, "linear_bwd_data"), (train_ops, "linear_wgrad"),
                          (train_ops, "subm_conv_bwd_data"), (ptv3_ops, "cpe_residual_ln"),
                          (ptv3_ops, "block_mlp"), (ptv3_ops, "subm_cpe_ln"), (ptv3_ops, "heads"),
                          (ptv3_ops, "window_attention_proj"), (ptv3_ops, "cpe_ln_qkv")]:
            fn = getattr(mod, name)
            self._saved.append((mod, name, fn))
            setattr(mod, name, self._wrap(name, fn))
        return self

    def _wrap(self, kind, fn):
        from splatformer_amd import ptv3_ops
        rec = self

        def wrapped(*args, **kw):
            if kind == "cpe_residual_ln" and not isinstance(args[0], ptv3_ops.SubmPartials):
                return fn(*args, **kw)  # (a LayerNorm, not part of the GEMM family)
            st = torch.cuda.current_stream()  # the stream libsfx launches on (_lib.stream())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            res = fn(*args, **kw)
            e1.record(st)
            fl, by, shape = _gemm_cost(kind, args, kw, res)
            rec.calls.append((kind, fl, by, shape, e0, e1))
            return res
        return wrapped

    def __exit__(self, *a):
        for mod, name, fn in self._saved:
            setattr(mod, name, fn)

    def summary(self):
        torch.cuda.synchronize()
        per = [(e0.elapsed_time(e1), kind, shape, fl() if callable(fl) else fl, by)
               for kind, fl, by, shape, e0, e1 in self.calls]
        return per


def roofline_probe(unit_fn, passes=3, dump=None):
    """achieved = algorithmic FLOP of every GEMM-family launch of one unit of work / their summed in-context
    durations; median over `passes` passes of the unit."""
    runs = []
    for _ in range(passes):
        torch.cuda.synchronize()
        with GemmTimer() as t:
            unit_fn()
        runs.append(t.summary())
    tot = [(sum(p[0] for p in r), r) for r in runs]
    tot.sort(key=lambda x: x[0])
    ms, per = tot[len(tot) // 2]
    if dump:
        with open(dump, "w") as f:
            for p in per:
                f.write(json.dumps({"kind": p[1], "shape": list(p[2]), "ms": round(p[0], 4),
                                    "tflops": round(p[3] / max(p[0], 1e-9) / 1e9, 2)}) + "\n")
    fl = sum(p[3] for p in per)
    by = sum(p[4] for p in per)
    achieved = fl / (ms * 1e-3) / 1e12
    top = max(per)
    # the family grew (round 3: + the fused MLP and the pair-sum LayerNorm); the pure-GEMM subset
    # (gemm_kernel / wgrad_kernel launches only) is the figure comparable with rounds 1-2
    pure = [p for p in per if p[1] not in ("block_mlp", "cpe_residual_ln", "subm_cpe_ln", "heads",
                                           "window_attention_proj", "cpe_ln_qkv")]
    pms, pfl = sum(p[0] for p in pure), sum(p[3] for p in pure)
    pure_tf = pfl / (pms * 1e-3) / 1e12 if pms > 0 else 0.0
    return {
        "bound": "mfma", "achieved": round(achieved, 2), "peak": SPLIT_PEAK_TFLOPS, "unit": "TFLOP/s",
        "frac": round(achieved / SPLIT_PEAK_TFLOPS, 4), "traffic": None,
        "algorithmic_bytes": int(by),
        "peak_basis": (f"fp32-equivalent ceiling of the fp16x2 split GEMM = dense fp16 MFMA {F16_MFMA_PEAK_TFLOPS:.0f}"
                       f" / 3 term products; exact-fp32 MFMA peak is {FP32_MFMA_PEAK_TFLOPS}"),
        "frac_of_fp32_mfma_peak": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4),
        "kernel": ("GEMM family (gemm_kernel: sfx_linear / sfx_subm_conv / training data-gradient GEMMs, fp32 "
                   "operands as power-of-two-scaled fp16x2 terms, 3 x v_mfma_f32_32x32x16_f16 per block, fp32 "
                   "accumulation; wgrad_kernel; mlp_kernel, the fused LN2 + fc1 + GELU + fc2 Block tail; "
                   "subm_cpe_ln_kernel, the SubM conv with its pair products summed on chip + the CPE LayerNorm "
                   "tail (C <= 128); heads_kernel, the six output MLPs; attn_proj_kernel, the window attention "
                   "fused with the output projection + residual (counted with its attention FLOP, 4 K C per point, "
                   "and its projection FLOP, 2 C^2 per point); cpe_ln_qkv_kernel, the SubM conv's pair sums + the CPE "
                   "and norm1 LayerNorms + the qkv projection (its 6 C^2 FLOP per point) at C <= 128; and "
                   "cpe_residual_ln4_kernel<.., true>, the "
                   "C >= 256 SubM conv's per-row sum of its stored pair products), "
                   "every launch of one unit of work incl. operand-maxima passes"),
        "timing": "HIP events around each launch on its stream, in the real launch sequence; median of "
                  f"{passes} passes",
        "launches": len(per), "gemm_ms_per_unit": round(ms, 3), "algorithmic_gflop_per_unit": round(fl / 1e9, 1),
        "top_launch": {"op": top[1], "M_N_K": list(top[2]), "ms": round(top[0], 4),
                       "tflops": round(top[3] / (top[0] * 1e-3) / 1e12, 2)},
        "pure_gemm": {"launches": len(pure), "ms_per_unit": round(pms, 3), "gflop_per_unit": round(pfl / 1e9, 1),
                      "achieved": round(pure_tf, 2), "frac": round(pure_tf / SPLIT_PEAK_TFLOPS, 4),
                      "kernels": "gemm_kernel + wgrad_kernel launches only (the rounds 1-2 family definition)"},
    }


# ---- HBM traffic from rocprofv3 PMC passes (child processes) -------------------------------------------------
def _pmc_pass(counter, argv, outdir, timeout_s=240):
    rp = shutil.which("rocprofv3")
    if rp is None:
        return None, "rocprofv3 not found"
    cmd = ["timeout", "-s", "KILL", str(timeout_s), rp, "--pmc", counter, "-d", outdir, "-o", "run",
           "--output-format", "csv", "--", sys.executable, os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env, cwd=ROOT)
    files = glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True)
    if r.returncode != 0 or not files:
        return None, f"rocprofv3 --pmc {counter}: rc {r.returncode}: {r.stdout.decode(errors='replace')[-300:]}"
    return files[0], None


def _per_unit(csv_path, counter):
    """Sum of `counter` over the GEMM-family dispatches between consecutive profile markers, per unit (the
    median unit); counters in KiB."""
    rows = []
    with open(csv_path) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter:
                continue
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    marks = [d for d, k, _ in rows if "profile_marker_kernel" in k]
    if len(marks) < 2:
        raise RuntimeError(f"{counter}: {len(marks)} profile markers in {csv_path}")
    units = []
    for a, b in zip(marks[:-1], marks[1:]):
        units.append(sum(v for d, k, v in rows if a < d < b and in_family(k)) * 1024.0)
    return statistics.median(units), len(units)


def measure_traffic(args):
    """Two PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs, MI355X_MICROARCH.md) of this bench in
    --profile-only --markers mode, 1 warm-up + 2 marked units; -> HBM bytes per unit of the GEMM family
    (2*FETCH_SIZE + WRITE_SIZE: gfx950 FETCH_SIZE counts half the bytes of wide reads), or (None, reason)."""
    argv = ["--config", args.config, "--n", str(args.n), "--res", f"{args.width}x{args.height}",
            "--views", str(args.views), "--sh", str(args.sh), "--batch", str(args.batch), "--steps", "2",
            "--warmup", "1", "--profile-only", "--markers", "--train-prec", args.train_prec]
    tmp = tempfile.mkdtemp(prefix="sfx_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        got = {}
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            path, err = _pmc_pass(counter, argv, os.path.join(tmp, counter))
            if path is None:
                return None, err
            got[counter] = _per_unit(path, counter)
        fetch, n_units = got["FETCH_SIZE"]
        write, _ = got["WRITE_SIZE"]
        return {"hbm_B": 2 * fetch + write, "fetch_B": 2 * fetch, "write_B": write, "units": n_units}, None
    except Exception as e:  # a profiler problem must not lose the bench line
        return None, f"traffic measurement failed: {e}"
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


# ---- CPU baseline (the oracle on the host cores) --------------------------------------------------------------
def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def _cgroup_cpus():
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            return max(1, int(float(q) / float(p)))
    except (OSError, ValueError):
        pass
    return None


def cpu_threads():
    """(threads used, affinity cores, cgroup CPU quota): all affinity cores, capped by the
    container's CPU quota when one is set (more threads than the quota only time-slice)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = _cgroup_cpus()
    return (min(aff, quota) if quota else aff), aff, quota


def _median_time(fn, repeats=3, warmup=True):
    if warmup:
        fn()
    ts = []
    for _ in range(repeats):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts), ts


def cpu_baseline(scene_cpu, cams_cpu, sd, cfg_kw, sample_n, n_total, views, sh):
    """The CPU oracle (oracle/, test infrastructure) on the same workload: FeaturePredictor forward on the
    first `sample_n` Gaussians + one view of that refined sample; 1 warm-up + median of 3 each, or one timed run
    each when the sample is >= 50k Gaussians (config B's whole scene: ~14 s + ~4 s, within the 10-30 s bound).
    When the sample is the whole scene (configs A, B) nothing is extrapolated except view 1 -> `views` views."""
    from oracle import ptv3_ref, render_ref
    threads, aff, quota = cpu_threads()
    torch.set_num_threads(threads)
    sub = {k: v[:sample_n].contiguous() for k, v in scene_cpu.items()}
    perms = [[0, 1, 2, 3]] * 5
    cfg = ptv3_ref.PTv3Config(in_channels=sd["backbone.backbone.embedding.0.weight"].shape[1], **cfg_kw)
    holder = {}

    def fwd():
        holder["out"], _ = ptv3_ref.feature_predictor_forward(sd, cfg, sub, perms, sh_degree=sh)

    big = sample_n >= 50_000
    reps = dict(repeats=1, warmup=False) if big else {}
    t_fwd, ts_fwd = _median_time(fwd, **reps)
    c2w = cams_cpu["camera_to_worlds"][0]
    t_view, ts_view = _median_time(lambda: render_ref.rasterize_gaussians_to_singleimg(holder["out"], c2w,
                                                                                       **cams_cpu), **reps)
    scale = n_total / sample_n
    t_scene = t_fwd * scale + views * t_view * scale
    whole = sample_n == n_total
    return {
        "value": round(views / t_scene, 5), "unit": "renders/s", "cores": threads, "kind": "port",
        "cpu_model": _cpu_model(), "affinity_cores": aff, "cgroup_cpu_quota": quota,
        "protocol": ("one timed run each (refine, one view): whole-scene runs of many seconds" if big else
                     "1 warm-up + median of 3 (refine and one view separately)"),
        "sample": (f"oracle FeaturePredictor fwd on {'all' if whole else 'the first'} {sample_n} of {n_total} "
                   f"Gaussians (median {t_fwd:.2f}s of {[round(t, 2) for t in ts_fwd]}) + 1 of {views} views of "
                   f"that refined {'scene' if whole else 'crop'} (median {t_view:.2f}s); "
                   + ("view time x " + str(views) if whole else
                      f"both scaled linearly by N ({scale:.1f}x) and the view time by {views}")),
    }


def cpu_baseline_train(scene_cpu, cams_cpu, sd0, sample_n, n_total, views, scenes_per_step):
    """The CPU oracle's train step on a bounded sample: refiner train-mode forward + autograd backward to the
    qkv parameters on a crop, plus one forward render of the refined crop (render backward not included);
    1 warm-up + median of 3."""
    from oracle import ptv3_ref, render_ref
    threads, aff, quota = cpu_threads()
    torch.set_num_threads(threads)
    sub = {k: v[:sample_n].contiguous() for k, v in scene_cpu.items()}
    perms = [[0, 1, 2, 3]] * 5
    holder = {}

    def step():
        sd = {k: v.clone() for k, v in sd0.items()}
        for k, v in sd.items():
            if "attn.qkv" in k:
                v.requires_grad_()
        out, _ = ptv3_ref.feature_predictor_forward(sd, ptv3_ref.PTv3Config(), sub, perms, train=True)
        loss = sum(v.abs().mean() for v in out.values())
        loss.backward()
        holder["out"] = {k: v.detach() for k, v in out.items()}

    big = sample_n >= 50_000
    reps = dict(repeats=1, warmup=False) if big else {}
    t_ref, ts = _median_time(step, **reps)
    c2w = cams_cpu["camera_to_worlds"][0]
    with torch.no_grad():
        t_view, _ = _median_time(lambda: render_ref.rasterize_gaussians_to_singleimg(holder["out"], c2w, **cams_cpu),
                                 **reps)
    scale = n_total / sample_n
    whole = sample_n == n_total
    t_step = scenes_per_step * (t_ref * scale + views * t_view * scale)
    return {
        "value": round(scenes_per_step * views / t_step, 6), "unit": "renders/s", "cores": threads, "kind": "port",
        "cpu_model": _cpu_model(), "affinity_cores": aff, "cgroup_cpu_quota": quota,
        "protocol": "one timed run each (whole-scene runs of many seconds)" if big else "1 warm-up + median of 3",
        "sample": (f"oracle FeaturePredictor train fwd+bwd (autograd, qkv grads) on {'all' if whole else 'the first'} "
                   f"{sample_n} of {n_total} Gaussians ({t_ref:.2f}s) + 1 forward view of that "
                   f"{'scene' if whole else 'crop'} ({t_view:.2f}s); "
                   + ("" if whole else f"scaled linearly by N ({scale:.1f}x); ")
                   + f"view time x {views} views, scene time x {scenes_per_step} scenes per step; "
                     "render backward not timed"),
    }


# ---- PSNR delta vs the oracle (eval configs) ---------------------------------------------------------------
def psnr_delta(model, scene, scene_cpu, cams, cams_cpu, sd_cpu, cfg_kw, sh, view=0):
    """the PSNR delta vs the oracle on the same inputs, on one view of the benchmarked scene --
    the HIP pipeline (refine + render) against the oracle pipeline (oracle refine with the same weights and
    order shuffles, oracle render), both scored as the reference's evaluation does (uint8 truncation,
    train.py:104-113; psnr on /255, utils/metrics.py:89-91) against the same target: the render of the
    unrefined input scene (synthetic data has no ground-truth photo).  Outside the timed region."""
    from oracle import gsplat_ref, ptv3_ref, render_ref
    from splatformer_amd.gs_render import rasterize_gaussians_to_singleimg
    threads, _, _ = cpu_threads()
    torch.set_num_threads(threads)
    t0 = time.perf_counter()
    with torch.no_grad():
        out = model([scene], [0])[0]
        perms = [list(p) for p in model.backbone.backbone.last_perms]
        c2w = cams["camera_to_worlds"][view]
        hip = rasterize_gaussians_to_singleimg(out, c2w, **cams)[0].cpu()
        gt = rasterize_gaussians_to_singleimg(scene, c2w, **cams)[0].cpu()
    cfg = ptv3_ref.PTv3Config(in_channels=sd_cpu["backbone.backbone.embedding.0.weight"].shape[1], **cfg_kw)
    if cfg.enable_flash:
        cfg.patch_size = 1024  # (the flash branch's patch, pointtransformer_v3.py:121-123)
    t1 = time.perf_counter()
    ref, _ = ptv3_ref.feature_predictor_forward(sd_cpu, cfg, scene_cpu, perms, sh_degree=sh)
    t2 = time.perf_counter()
    orc, _ = render_ref.rasterize_gaussians_to_singleimg(ref, cams_cpu["camera_to_worlds"][view], **cams_cpu)
    t3 = time.perf_counter()
    p_hip = float(gsplat_ref.psnr_u8(hip[None], gt[None]))
    p_orc = float(gsplat_ref.psnr_u8(orc[None], gt[None]))
    return {"psnr_delta_db": round(p_hip - p_orc, 7), "view": view, "psnr_hip_db": round(p_hip, 5),
            "psnr_oracle_db": round(p_orc, 5), "max_abs_pixel_diff": float((hip - orc).abs().max()),
            "target": "render of the unrefined input scene (same view)",
            "oracle": f"oracle/ptv3_ref + oracle/render_ref, whole scene, {threads} threads, "
                      f"{time.perf_counter() - t0:.1f}s",
            "_oracle_times": (t2 - t1, t3 - t2)}  # (whole-scene refine, one view): the CPU baseline's legs


def cpu_baseline_from_psnr(psnr, n_total, views):
    """The CPU baseline of an eval config from the PSNR leg's own oracle runs -- the whole-scene oracle refine and
    its render of one view (one timed run each) -- instead of timing the same work a second time.  Nothing is
    extrapolated in N; the one view's time stands for each of the `views` views (same camera ring, same scene)."""
    t_ref, t_view = psnr.pop("_oracle_times")
    threads, aff, quota = cpu_threads()
    return {
        "value": round(views / (t_ref + views * t_view), 5), "unit": "renders/s", "cores": threads, "kind": "port",
        "cpu_model": _cpu_model(), "affinity_cores": aff, "cgroup_cpu_quota": quota,
        "protocol": "one timed run each (whole-scene runs of many seconds), shared with the PSNR leg",
        "sample": (f"oracle FeaturePredictor fwd on all {n_total} Gaussians ({t_ref:.2f}s) + 1 of {views} views of the "
                   f"refined scene ({t_view:.2f}s); view time x {views}"),
    }


# ---- main -----------------------------------------------------------------------------------------------------
def main(argv=None):
    args = parse(argv)
    if needs_launch(args.gpus):  # before anything touches the GPU
        sys.exit(subprocess.call(launch_cmd(args.gpus, sys.argv[1:] if argv is None else argv, _free_port())))
    from splatformer_amd import dist as sdist
    rank, world, local_rank = sdist.env_rank()
    world_size_check(args.gpus, world)
    if args.dry_launch:  # the launcher's CPU test: report the rank layout, touch no GPU
        print(json.dumps({"rank": rank, "world": world, "local_rank": local_rank}), flush=True)
        return
    dev = torch.device("cuda", local_rank if world > 1 else 0)
    torch.cuda.set_device(dev)
    multi = sdist.init("nccl")  # RCCL: barrier + max-over-ranks timing; config D adds the gradient all-reduce

    from splatformer_amd import _lib
    from splatformer_amd.feature_predictor import FeaturePredictor
    from splatformer_amd.gs_render import rasterize_gaussians_to_multiimgs
    from splatformer_amd.scenes import make_cameras, make_scene, to_device
    _lib.load()
    train = args.config in ("C", "D")
    cams_cpu = make_cameras(args.width, args.height, n_views=args.views)
    cams = to_device(cams_cpu, dev)
    bk = dict(DEPTH1) if args.config == "A" else {}
    if args.flash:
        bk["enable_flash"] = True
    torch.manual_seed(0)
    model = FeaturePredictor(sh_degree=args.sh, zeroinit=False, backbone_kwargs=bk).eval()
    sd_cpu = {k: v.detach().clone() for k, v in model.state_dict().items()}
    model = model.to(dev)

    if not train:
        scene_cpu = make_scene(args.n, sh_degree=args.sh, seed=rank)
        scene = to_device(scene_cpu, dev)

        def step():
            out = model([scene], [rank])[0]
            rgbs, alphas = rasterize_gaussians_to_multiimgs(out, cams)
            return rgbs

        def unit():  # the GEMM family's unit of work: one refine
            model.refine_packed(scene)
        renders_per_step = args.views
    else:
        from splatformer_amd.train import Trainer
        n_sc = args.batch
        scenes_cpu = [make_scene(args.n, sh_degree=args.sh, seed=rank * n_sc + i) for i in range(n_sc)]
        scene_cpu = scenes_cpu[0]
        scenes = [to_device(sc, dev) for sc in scenes_cpu]
        with torch.no_grad():  # synthetic targets: the input scenes' own renders
            gts = [rasterize_gaussians_to_multiimgs(sc, cams)[0] for sc in scenes]
        group = torch.distributed.group.WORLD if multi else None
        tr = Trainer(model, accumulate_step=(n_sc if args.config == "D" else 1), group=group,
                     generator=torch.Generator(device=dev).manual_seed(rank), precision=args.train_prec)

        if args.config == "C":
            def step():
                tr.micro_step(scenes, [cams] * n_sc, gts)
                tr.optimizer_step()
        else:
            def step():
                for i in range(n_sc):
                    tr.micro_step([scenes[i]], [cams], [gts[i]])
                tr.optimizer_step()

        def unit():  # one training micro-step of one scene: train forward + backward (no optimiser step)
            tr.micro_step([scenes[0]], [cams], [gts[0]])
        renders_per_step = args.views * n_sc

    marker = (lambda i: _lib.call("sfx_profile_marker", i, _lib.stream())) if args.markers else (lambda i: None)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    sdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        marker(i)
        step()
    marker(args.steps)
    torch.cuda.synchronize()
    sdist.barrier()
    t1 = time.perf_counter()
    elapsed = sdist.max_over_ranks(t1 - t0, device=dev)
    value = renders_per_step * args.steps * world / elapsed
    # the timed steps' results are consumed here (outside the timed region): the refines' deferred pooled-count
    # checks and every look-back scan / radix pass of the run must have been exact, or the line is not printed
    if not train:
        model.check_refine()
    _lib.check_lookback("bench.py timed steps")

    roof = None
    if not args.profile_only:
        if not train:
            model.eval()
        roof = roofline_probe(unit, dump=args.gemm_calls if rank == 0 else None)
        if rank == 0 and world == 1 and not args.no_traffic:
            tr_res, err = measure_traffic(args)
            if tr_res is not None:
                roof["traffic"] = tr_res["hbm_B"]
                roof["traffic_detail"] = {**tr_res, "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes run "
                                                               "by bench.py (2*FETCH + WRITE, per unit, median)"}
                roof["traffic_over_algorithmic"] = round(tr_res["hbm_B"] / max(1, roof["algorithmic_bytes"]), 3)
            else:
                roof["traffic_note"] = err
    psnr = None
    if rank == 0 and world == 1 and not train and not args.no_psnr and not args.profile_only:
        psnr = psnr_delta(model, scene, scene_cpu, cams, cams_cpu, sd_cpu, bk, args.sh)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.profile_only:
        # the whole scene by default (no extrapolation in N); --cpu-sample bounds it for quick runs
        sample = min(args.cpu_sample or args.n, args.n)
        if train:
            cpu = cpu_baseline_train(scene_cpu, cams_cpu, sd_cpu, sample, args.n, args.views, args.batch)
        elif psnr is not None and sample == args.n and not args.flash:
            cpu = cpu_baseline_from_psnr(psnr, args.n, args.views)
        else:
            cpu = cpu_baseline(scene_cpu, cams_cpu, sd_cpu, bk, sample, args.n, args.views, args.sh)
    if psnr is not None:
        psnr.pop("_oracle_times", None)

    if rank == 0:
        res = f"{args.width}x{args.height}"
        unit_name = "one training micro-step (train fwd + bwd of one scene)" if train else "one refine"
        if args.config == "C":
            workload = (f"C: batch {args.batch} scenes x {args.n} Gaussians SH{args.sh}, train-mode refine + "
                        f"{args.views} views {res} each, image-L1 fwd+bwd, clip + Adam (attn.qkv)")
            par = f"scene-dp{world}" if world > 1 else "single-gpu"
        elif args.config == "D":
            workload = (f"D: DDP, per rank {args.batch} micro-steps x 1 scene ({args.n} GS SH{args.sh}, {args.views} "
                        f"views {res}) per optimiser step, RCCL grad all-reduce + SyncBN")
            par = f"ddp{world}-accum{args.batch}"
        else:
            depth = "depth-1 PTv3" if args.config == "A" else "full PTv3 (ptv3_base)"
            workload = (f"{args.config}: {args.n} Gaussians SH{args.sh}, {depth} + heads, "
                        f"{args.views} views {res}, forward")
            par = f"scene-dp{world}"
        if roof is not None:
            roof["unit_of_work"] = unit_name
        line = {
            "metric": "refined renders/sec (100k GS, 800x800) at 1/2/4/8 MI355X; PSNR vs ref" if args.config == "B"
            else f"refined renders/sec (config {args.config})",
            "value": round(value, 3),
            "unit": "renders/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": ("fp16-autocast-class (refiner GEMMs: leading fp16 term product, fp32 accumulation; "
                      "--train-prec amp)") if train and args.train_prec == "amp" else "fp32",
            "data": f"synthetic (seeded {args.n}-Gaussian scene(s) per rank, random-init ptv3_base weights)",
            "config": {"workload": workload, "scenes_per_step": (args.batch if train else 1) * world,
                       "views_per_scene": args.views, "parallelism": par,
                       "attention": "flash (K=1024 varlen)" if args.flash else "non-flash (K=128, ptv3_base.gin:27)"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "psnr": psnr,
        }
        print(json.dumps(line), flush=True)
    if multi:
        sdist.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
