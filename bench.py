"""Benchmark of the SplatFormer hot path on MI355X (BASELINE.json configs).

Default (the driver's line) = config B: refined renders/sec on 100k-Gaussian x 800x800 scenes.  One step =
one scene per rank: FeaturePredictor forward (full ptv3_base PTv3 + heads, fp32) over 100k Gaussians, then
the 9 OOD test views (800x800) of the refined Gaussians through the gsplat-v0.1.11-semantics renderer -- the
reference's evaluation() hot loop (train.py:86-100).  Synthetic seeded scene and random-init weights of the
ptv3_base architecture (no datasets/checkpoints offline).  Multi-GPU: one process per GPU, one scene per
rank (weak scaling, no collective on the data path; barrier + max-over-ranks timing only).

--config C: training -- a step = a batch of 8 scenes (100k GS, SH1), each refined in train mode, rendered to
  4 training views (800x800), image-L1 loss, backward through renderer + refiner, then clip + Adam
  (train.py:236-303); renders/s = 8*4 / step time.
--config D: DDP training under torchrun -- per rank one scene per micro-step, 4 micro-steps per optimiser
  step (accumulate 4), RCCL all-reduce of the gradient bucket + SyncBatchNorm; a step = one optimiser step.
--config E: 500k Gaussians, SH3, 1920x1080, 9 views, forward (HBM-bound stress).

Prints ONE JSON line (rank 0) with `roofline` for the dominant kernel (the fp32 MFMA GEMM, every launch of
one refine replayed between HIP events on the launch stream) and `cpu_baseline` (the CPU oracle on a
bounded sample, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
F16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense fp16 / bf16 MFMA (no sparsity)
# The GEMM computes fp32-accurate products as three fp16 term products (fp16x2 split operands, gemm.hip): its
# fp32-equivalent ceiling is the dense fp16 peak / 3.
SPLIT_PEAK_TFLOPS = round(F16_MFMA_PEAK_TFLOPS / 3, 1)
# rocprofv3 FETCH_SIZE / WRITE_SIZE passes over this bench (tools/traffic_summary.py), committed per round
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "r01_traffic_f16x2.json")
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=["B", "C", "D", "E"], default="B")
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--res", type=str, default=None, help="W or WxH")
    ap.add_argument("--views", type=int, default=None)
    ap.add_argument("--sh", type=int, default=None)
    ap.add_argument("--batch", type=int, default=None, help="scenes per step (C) / micro-steps (D)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=20_000, help="Gaussians in the CPU-oracle sample")
    ap.add_argument("--profile-only", action="store_true", help="skip roofline probe and CPU baseline")
    a = ap.parse_args()
    dflt = {"B": (100_000, "800", 9, 1, 1), "C": (100_000, "800", 4, 1, 8), "D": (100_000, "800", 4, 1, 4),
            "E": (500_000, "1920x1080", 9, 3, 1)}[a.config]
    a.n = a.n if a.n is not None else dflt[0]
    res = a.res if a.res is not None else dflt[1]
    a.width, a.height = (int(res.split("x")[0]), int(res.split("x")[1])) if "x" in res else (int(res), int(res))
    a.views = a.views if a.views is not None else dflt[2]
    a.sh = a.sh if a.sh is not None else dflt[3]
    a.batch = a.batch if a.batch is not None else dflt[4]
    return a


class GemmRecorder:
    """Records the GEMM-kernel launches (sfx_linear / sfx_subm_conv) of one refine pass."""

    def __init__(self):
        self.calls = []

    def __enter__(self):
        from splatformer_amd import ptv3_ops
        self._lin, self._conv, self._grp = ptv3_ops.linear, ptv3_ops.subm_conv, ptv3_ops.grouped_linear
        rec = self

        def lin(x, weight, bias=None, **kw):
            res = rec._lin(x, weight, bias, **kw)
            out = res[0] if isinstance(res, tuple) else res
            M = out.shape[0]
            N, K = weight.shape
            kw2 = dict(kw)
            kw2["out"] = torch.empty_like(out) if kw.get("out") is None else torch.empty_like(kw["out"])
            rec.calls.append(("linear", 2.0 * M * N * K, lambda: rec._lin(x, weight, bias, **kw2), (M, N, K)))
            return res

        def conv(x, smap, weight, bias, out=None, **kw):
            o = rec._conv(x, smap, weight, bias, out=out, **kw)
            n, cin = x.shape
            cout = weight.shape[0]
            scratch = torch.empty_like(o)
            fl = 2.0 * (n + smap.num_pairs) * cin * cout
            rec.calls.append(("subm_conv", fl, lambda: rec._conv(x, smap, weight, bias, out=scratch, **kw),
                              (n, cout, cin)))
            return o

        def grp(x, weight, bias, groups, **kw):
            res = rec._grp(x, weight, bias, groups, **kw)
            out = res[0] if isinstance(res, tuple) else res
            G, N, K = weight.shape
            scratch = torch.empty_like(out)
            rec.calls.append(("grouped_linear", 2.0 * x.shape[0] * G * N * K,
                              lambda: rec._grp(x, weight, bias, groups, **dict(kw, out=scratch)),
                              (x.shape[0], G * N, K)))
            return res

        ptv3_ops.linear, ptv3_ops.subm_conv, ptv3_ops.grouped_linear = lin, conv, grp
        return self

    def __exit__(self, *a):
        from splatformer_amd import ptv3_ops
        ptv3_ops.linear, ptv3_ops.subm_conv, ptv3_ops.grouped_linear = self._lin, self._conv, self._grp


def roofline_probe(model, scene, reps=5):
    """Replay every GEMM-kernel launch of one refine pass between HIP events (on the launch stream):
    achieved = algorithmic FLOP of all launches / summed average launch time."""
    with GemmRecorder() as rec:
        model.refine_packed(scene)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    tot_fl, tot_ms, per = 0.0, 0.0, []
    for kind, fl, fn, shape in rec.calls:
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        tot_fl += fl
        tot_ms += ms
        per.append((ms, kind, shape, fl))
    achieved = tot_fl / (tot_ms * 1e-3) / 1e12
    top = max(per)
    traffic = None
    try:  # measured HBM bytes of the same launches (PMC passes, per scene), see TRAFFIC_FILE
        with open(TRAFFIC_FILE) as f:
            traffic = json.load(f)["per_scene"]["gemm_kernel"]["hbm_B"]
    except (OSError, KeyError, ValueError):
        pass
    return {
        "bound": "mfma", "achieved": round(achieved, 2), "peak": SPLIT_PEAK_TFLOPS, "unit": "TFLOP/s",
        "frac": round(achieved / SPLIT_PEAK_TFLOPS, 4), "traffic": traffic,
        "traffic_unit": "HBM bytes per scene (all GEMM launches; 2*FETCH_SIZE + WRITE_SIZE, " +
                        os.path.relpath(TRAFFIC_FILE, ROOT) + ")",
        "peak_basis": (f"fp32-equivalent ceiling of the fp16x2 split GEMM = dense fp16 MFMA {F16_MFMA_PEAK_TFLOPS:.0f}"
                       f" / 3 term products; exact-fp32 MFMA peak is {FP32_MFMA_PEAK_TFLOPS}"),
        "frac_of_fp32_mfma_peak": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4),
        "kernel": ("gemm_kernel (sfx_linear / sfx_subm_conv: fp32 operands scaled by powers of two and split into "
                   "2 fp16 terms, 3 x v_mfma_f32_32x32x16_f16 per block, fp32 accumulation; K < 64: exact fp32 "
                   "MFMA), all launches of one scene (incl. their operand-maxima passes)"),
        "launches": len(per), "gemm_ms_per_scene": round(tot_ms, 3),
        "algorithmic_gflop_per_scene": round(tot_fl / 1e9, 1),
        "top_launch": {"op": top[1], "M_N_K": list(top[2]), "avg_ms": round(top[0], 4),
                       "tflops": round(top[3] / (top[0] * 1e-3) / 1e12, 2)},
    }


def cpu_baseline(scene_cpu, cams_cpu, model_cpu_sd, sample_n, n_total, views, threads):
    """The CPU oracle (oracle/) on a bounded sample of the workload (test infrastructure, not the product)."""
    from oracle import ptv3_ref, render_ref
    torch.set_num_threads(threads)
    idx = torch.arange(sample_n)
    sub = {k: v[idx].contiguous() for k, v in scene_cpu.items()}
    perms = [[0, 1, 2, 3]] * 5
    t0 = time.perf_counter()
    out, _ = ptv3_ref.feature_predictor_forward(model_cpu_sd, ptv3_ref.PTv3Config(), sub, perms)
    t_fwd = time.perf_counter() - t0
    c2w = cams_cpu["camera_to_worlds"][0]
    t0 = time.perf_counter()
    render_ref.rasterize_gaussians_to_singleimg(out, c2w, **cams_cpu)
    t_view = time.perf_counter() - t0
    scale = n_total / sample_n
    t_scene = t_fwd * scale + views * t_view * scale
    return {
        "value": round(views / t_scene, 5), "unit": "renders/s", "cores": threads, "kind": "port",
        "sample": (f"oracle FeaturePredictor fwd on the first {sample_n} of {n_total} Gaussians ({t_fwd:.2f}s) + 1 of "
                   f"{views} views of that refined crop ({t_view:.2f}s); both scaled linearly by N "
                   f"({scale:.1f}x) and the view time by {views}"),
    }


def _threads():
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    return max(1, min(16, aff))


def cpu_baseline_train(scene_cpu, cams_cpu, model_cpu_sd, sample_n, n_total, views, scenes_per_step, threads):
    """The CPU oracle's train step on a bounded sample: refiner train-mode forward + autograd backward to the
    qkv parameters on a crop, plus one forward render of the refined crop (render backward not included)."""
    from oracle import ptv3_ref, render_ref
    torch.set_num_threads(threads)
    sub = {k: v[:sample_n].contiguous() for k, v in scene_cpu.items()}
    perms = [[0, 1, 2, 3]] * 5
    sd = {k: v.clone() for k, v in model_cpu_sd.items()}
    for k, v in sd.items():
        if "attn.qkv" in k:
            v.requires_grad_()
    t0 = time.perf_counter()
    out, _ = ptv3_ref.feature_predictor_forward(sd, ptv3_ref.PTv3Config(), sub, perms, train=True)
    loss = sum(v.abs().mean() for v in out.values())
    loss.backward()
    t_ref = time.perf_counter() - t0
    c2w = cams_cpu["camera_to_worlds"][0]
    t0 = time.perf_counter()
    with torch.no_grad():
        render_ref.rasterize_gaussians_to_singleimg({k: v.detach() for k, v in out.items()}, c2w, **cams_cpu)
    t_view = time.perf_counter() - t0
    scale = n_total / sample_n
    t_step = scenes_per_step * (t_ref * scale + views * t_view * scale)
    return {
        "value": round(scenes_per_step * views / t_step, 6), "unit": "renders/s", "cores": threads, "kind": "port",
        "sample": (f"oracle FeaturePredictor train fwd+bwd (autograd, qkv grads) on the first {sample_n} of {n_total} "
                   f"Gaussians ({t_ref:.2f}s) + 1 forward view of that crop ({t_view:.2f}s); scaled by N ({scale:.1f}x), "
                   f"views ({views}) and scenes/step ({scenes_per_step}); render backward not timed"),
    }


def main():
    args = parse()
    from splatformer_amd import dist as sdist
    rank, world, local_rank = sdist.env_rank()
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
    torch.manual_seed(0)
    model = FeaturePredictor(sh_degree=args.sh, zeroinit=False).eval()
    sd_cpu = {k: v.detach().clone() for k, v in model.state_dict().items()}
    model = model.to(dev)

    if not train:
        scene_cpu = make_scene(args.n, sh_degree=args.sh, seed=rank)
        scene = to_device(scene_cpu, dev)

        def step():
            out = model([scene], [rank])[0]
            rgbs, alphas = rasterize_gaussians_to_multiimgs(out, cams)
            return rgbs
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
                     generator=torch.Generator(device=dev).manual_seed(rank))

        if args.config == "C":
            def step():
                tr.micro_step(scenes, [cams] * n_sc, gts)
                tr.optimizer_step()
        else:
            def step():
                for i in range(n_sc):
                    tr.micro_step([scenes[i]], [cams], [gts[i]])
                tr.optimizer_step()
        renders_per_step = args.views * n_sc

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    sdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    sdist.barrier()
    t1 = time.perf_counter()
    elapsed = sdist.max_over_ranks(t1 - t0, device=dev)
    value = renders_per_step * args.steps * world / elapsed

    roof = None
    if not args.profile_only:
        model.eval()
        roof = roofline_probe(model, to_device(scene_cpu, dev))
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.profile_only:
        sample = min(args.cpu_sample, args.n)
        if train:
            cpu = cpu_baseline_train(scene_cpu, cams_cpu, sd_cpu, sample, args.n, args.views, args.batch, _threads())
        else:
            cpu = cpu_baseline(scene_cpu, cams_cpu, sd_cpu, sample, args.n, args.views, _threads())

    if rank == 0:
        res = f"{args.width}x{args.height}"
        if args.config == "C":
            workload = (f"C: batch {args.batch} scenes x {args.n} Gaussians SH{args.sh}, train-mode refine + "
                        f"{args.views} views {res} each, image-L1 fwd+bwd, clip + Adam (attn.qkv)")
            par = "single-gpu"
        elif args.config == "D":
            workload = (f"D: DDP, per rank {args.batch} micro-steps x 1 scene ({args.n} GS SH{args.sh}, {args.views} "
                        f"views {res}) per optimiser step, RCCL grad all-reduce + SyncBN")
            par = f"ddp{world}-accum{args.batch}"
        else:
            workload = (f"{args.config}: {args.n} Gaussians SH{args.sh}, full PTv3 (ptv3_base) + heads, "
                        f"{args.views} views {res}, forward")
            par = f"scene-dp{world}"
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
            "dtype": "fp32",
            "data": f"synthetic (seeded {args.n}-Gaussian scene(s) per rank, random-init ptv3_base weights)",
            "config": {"workload": workload, "scenes_per_step": (args.batch if train else 1) * world,
                       "views_per_scene": args.views, "parallelism": par},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if multi:
        sdist.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
