"""Config D's optimiser-step semantics on one GPU: train-on-objaverse gpux8-accum4 is
reference train.py:227-303 under DDP + SyncBatchNorm (train.py:404, :413) -- every rank runs `accumulate_step`
micro-steps of one scene each (loss / accumulate_step, train.py:286), DDP averages the accumulated gradients over
the ranks, then clip_grad_norm_(2.0) and Adam(lr 3e-5, eps 1e-15) on the attn.qkv parameters
(utils/optimizers.py:46-52, configs/train/default.gin).

Here: 2 ranks (gloo, both on cuda:0; RCCL over >1 GPU is the driver's 8-GPU run), `Trainer(accumulate_step=4)`,
4 different scenes per rank, each micro-step the full step of config C (train-mode refine, render of 4 views
through the gsplat-compatible autograd path, image L1, backward through renderer and refiner).  The oracle
replays it: micro-step i is ONE train forward over the two ranks' i-th scenes as a 2-scene batch (its
BatchNorms see both scenes -- SyncBatchNorm's statistics of that micro-step), the upstream gradient of the
refined records = what HIP's renderer produced (the render backward itself is held to the oracle by
tests/test_gpu_config_c.py), the heads' ReLU active sets, DropPath masks and order shuffles replayed.

Checked:
* the averaged bucket == (1/world) sum_i grad of micro-step i's batch loss: as close to the fp64 oracle as
  the fp32 oracle is (2x + 1e-5);
* the BatchNorm running statistics after the 4 SyncBN micro-steps (momentum 0.01 each), rel <= 1e-5;
* the optimiser step: HIP's clip + Adam == torch.nn.utils.clip_grad_norm_ + torch.optim.Adam applied to the same
  averaged bucket (rel <= 1e-6); against Adam on the fp64 oracle's gradient every updated weight agrees to
  1e-2 lr except where the fp64 gradient itself is within 1e-3 of its rms of zero (a first Adam step is
  lr * sign(g): an element whose gradient is rounding noise may take either sign), and such disagreements are
  at most 1.01x (+1) as many as the fp32 oracle's own;
* the next micro-step's train forward on the updated weights vs the oracle's on its own updated weights:
  refined residual rel L2 <= 1e-5.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

WORLD, ACCUM, VIEWS, RES = 2, 4, 4, 96
SIZES = [[3000, 2600, 3400, 2800, 3100], [2700, 3300, 2500, 3200, 2900]]  # [rank][micro-step]; step 4 = next fwd
PERMS = [[[1, 0, 3, 2], [2, 3, 0, 1], [0, 1, 2, 3], [3, 2, 1, 0], [1, 3, 0, 2]],
         [[0, 1, 2, 3], [1, 2, 3, 0], [3, 0, 2, 1], [2, 1, 0, 3], [0, 3, 1, 2]],
         [[3, 2, 1, 0], [0, 1, 2, 3], [1, 0, 3, 2], [2, 0, 3, 1], [3, 1, 2, 0]],
         [[2, 3, 0, 1], [3, 0, 1, 2], [0, 2, 1, 3], [1, 3, 2, 0], [2, 1, 3, 0]],
         [[1, 2, 0, 3], [2, 0, 3, 1], [3, 1, 0, 2], [0, 3, 2, 1], [1, 0, 2, 3]]]
FEATS = ["means", "scales", "opacities", "quats", "features_dc", "features_rest"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scene(rank, i):
    from splatformer_amd.scenes import make_scene
    return make_scene(SIZES[rank][i], 1, seed=300 + 10 * i + rank)


def _model():
    from splatformer_amd.feature_predictor import FeaturePredictor
    torch.manual_seed(0)
    return FeaturePredictor(sh_degree=1, zeroinit=False)


def _worker(rank, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD))
    try:
        import torch.distributed as tdist
        from splatformer_amd import gs_render
        from splatformer_amd import train as strain
        from splatformer_amd.scenes import make_cameras, to_device
        from test_gpu_train import RecordingMasks
        tdist.init_process_group("gloo", rank=rank, world_size=WORLD)
        dev = torch.device("cuda", 0)
        model = _model().to(dev)
        tr = strain.Trainer(model, accumulate_step=ACCUM, group=tdist.group.WORLD)
        assert (tr.lr, tr.eps, tr.clip) == (3e-5, 1e-15, 2.0)
        W = model.width
        cap = {"relu": [], "packed": [], "d_packed": [], "masks": [], "perms": []}
        orig_refine, orig_backward, orig_reduce = strain.refine_train, strain.refine_backward, strain.allreduce_mean_

        def refine(fp, gs, masks, perms=None, group=None):
            packed, tape = orig_refine(fp, gs, masks, perms=perms, group=group)
            cap["relu"].append({f: [(h[:, g * W:(g + 1) * W] > 0).cpu().numpy() for h in tape["hs"]]
                                for g, f in enumerate(fp.output_features)})
            cap["packed"].append(packed.detach().cpu().numpy())
            cap["perms"].append([list(p) for p in fp.backbone.backbone.last_perms])
            return packed, tape

        def backward(fp, tape, d_packed):
            cap["d_packed"].append(d_packed.detach().cpu().numpy())
            return orig_backward(fp, tape, d_packed)

        def reduce(flat, group=None):
            out = orig_reduce(flat, group)
            cap["bucket"] = flat.detach().cpu().numpy().copy()
            return out

        strain.refine_train, strain.refine_backward, strain.allreduce_mean_ = refine, backward, reduce
        cams = to_device(make_cameras(RES, RES, n_views=VIEWS), dev)
        for i in range(ACCUM):
            gs = to_device(_scene(rank, i), dev)
            with torch.no_grad():
                gts = [g.clone() for g in gs_render.rasterize_gaussians_to_multiimgs(gs, cams)[0]]
            masks = RecordingMasks(500 + 10 * i + rank)
            tr.step([gs], [cams], [gts], masks=masks, perms=PERMS[i])
            cap["masks"].append({k: v.numpy() for k, v in masks.masks.items()})
            if i < ACCUM - 1:
                assert float(tr.flat_grad.abs().max()) > 0 and "bucket" not in cap  # still accumulating
        assert tr.step_count == 1 and float(tr.flat_grad.abs().max()) == 0.0
        cap["norm"] = float(tr.last_norm)
        sd = model.state_dict()
        cap["running"] = {k: v.cpu().numpy() for k, v in sd.items() if "running_" in k}
        cap["qkv"] = {k: p.detach().cpu().numpy() for k, p in model.named_parameters() if "attn.qkv" in k}
        # the next micro-step's train forward on the updated weights
        masks = RecordingMasks(900 + rank)
        strain.refine_train = orig_refine
        packed, _ = strain.refine_train(model, to_device(_scene(rank, ACCUM), dev), masks, perms=PERMS[ACCUM],
                                        group=tdist.group.WORLD)
        cap["next_packed"] = packed.cpu().numpy()
        cap["next_masks"] = {k: v.numpy() for k, v in masks.masks.items()}
        torch.cuda.synchronize()
        q.put((rank, cap))
        tdist.barrier()
    finally:
        if torch.distributed.is_initialized():
            torch.distributed.destroy_process_group()


@pytest.fixture(scope="module")
def ranks(device):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=600) for _ in range(WORLD)), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    caps = [c for _, c in res]
    assert (caps[0]["bucket"] == caps[1]["bucket"]).all()  # every rank holds the same averaged bucket
    for k in caps[0]["qkv"]:
        assert (caps[0]["qkv"][k] == caps[1]["qkv"][k]).all()  # ... and the same updated weights
    return caps


def _batch(i):
    """The ranks' micro-step-i scenes as one 2-scene batch (concatenated attributes, offsets)."""
    scenes = [_scene(r, i) for r in range(WORLD)]
    gs = {k: torch.cat([s[k] for s in scenes]) for k in scenes[0]}
    counts = [s["means"].shape[0] for s in scenes]
    return gs, counts


def _oracle_forward(sd, gs, counts, perms, masks, relu, dtype):
    from oracle import ptv3_ref
    data = ptv3_ref.batchify({k: v.to(dtype) for k, v in gs.items()})
    data["offset"] = torch.tensor(counts).cumsum(0)
    point = ptv3_ref.ptv3_forward(sd, ptv3_ref.PTv3Config(), data, perms, prefix="backbone.backbone.", train=True,
                                  masks={k: m.to(dtype) for k, m in masks.items()})
    out = ptv3_ref.heads_forward(sd, point.feat, data["feat"], {k: v.to(dtype) for k, v in gs.items()},
                                 relu_masks=relu)
    n = sum(counts)
    return torch.cat([out[f].reshape(n, -1) for f in FEATS], 1)


def _cat_masks(dicts):
    return {k: torch.cat([torch.from_numpy(d[k]) for d in dicts]) for k in dicts[0]}


def _oracle_accum(caps, dtype):
    """sum_i grad(micro-step i's 2-scene batch loss) / world, with the running statistics after the 4 steps."""
    sd0 = _model().state_dict()
    names = [k for k, _ in _model().named_parameters() if "attn.qkv" in k]
    batches = [_batch(i) for i in range(ACCUM)]  # (fp32 scenes: make_scene follows the default dtype)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(dtype)
    try:
        sd = {k: (v.to(dtype) if v.is_floating_point() else v).clone() for k, v in sd0.items()}
        for k in names:
            sd[k].requires_grad_()
        for i in range(ACCUM):
            assert caps[0]["perms"][i] == caps[1]["perms"][i] == PERMS[i]
            gs, counts = batches[i]
            masks = _cat_masks([c["masks"][i] for c in caps])
            relu = {f: [torch.cat([torch.from_numpy(c["relu"][i][f][li]) for c in caps])
                        for li in range(len(caps[0]["relu"][i][f]))] for f in caps[0]["relu"][i]}
            rp = _oracle_forward(sd, gs, counts, PERMS[i], masks, relu, dtype)
            d = torch.cat([torch.from_numpy(c["d_packed"][i]) for c in caps]).to(dtype)
            (rp * d).sum().backward()
    finally:
        torch.set_default_dtype(prev)
    grads = torch.cat([sd[k].grad.double().reshape(-1) for k in names]) / WORLD
    return sd, names, grads


@pytest.fixture(scope="module")
def oracle32(ranks):
    return _oracle_accum(ranks, torch.float32)


@pytest.fixture(scope="module")
def oracle64(ranks):
    return _oracle_accum(ranks, torch.float64)


def test_config_d_accumulated_bucket(ranks, oracle32, oracle64):
    from test_gpu_ptv3 import rel_l2
    hip = torch.from_numpy(ranks[0]["bucket"]).double()
    g32, g64 = oracle32[2], oracle64[2]
    e_hip, e_ref = rel_l2(hip, g64), rel_l2(g32, g64)
    print(f"\n[config D, 2 ranks x accum 4] averaged bucket to fp64: HIP {e_hip:.2e}, fp32 oracle {e_ref:.2e}")
    assert e_hip <= 2.0 * e_ref + 1e-5


def test_config_d_running_stats(ranks, oracle32):
    from test_gpu_ptv3 import rel_l2
    sd = oracle32[0]
    run = ranks[0]["running"]
    assert run
    for k, v in run.items():
        assert rel_l2(torch.from_numpy(v), sd[k].detach()) < 1e-5, k
        assert (v == ranks[1]["running"][k]).all(), k  # SyncBN: both ranks hold the same statistics


def _adam_update(w0, g, steps=1):
    """clip_grad_norm_(2.0) + torch.optim.Adam(lr 3e-5, eps 1e-15) on fp64 copies -> updated weights."""
    ps = [torch.nn.Parameter(w.clone().double()) for w in w0]
    off = 0
    for p in ps:
        p.grad = g[off:off + p.numel()].view_as(p).clone().double()
        off += p.numel()
    torch.nn.utils.clip_grad_norm_(ps, 2.0)
    opt = torch.optim.Adam(ps, lr=3e-5, eps=1e-15)
    opt.step()
    return torch.cat([p.detach().reshape(-1) for p in ps])


def test_config_d_optimizer_step(ranks, oracle32, oracle64):
    from test_gpu_ptv3 import rel_l2
    _, names, g64 = oracle64
    g32 = oracle32[2]
    sd0 = _model().state_dict()
    w0 = [sd0[k] for k in names]
    hip_w = torch.cat([torch.from_numpy(ranks[0]["qkv"][k]).double().reshape(-1) for k in names])
    bucket = torch.from_numpy(ranks[0]["bucket"]).double()
    # the norm HIP clipped with == the bucket's L2 norm
    assert abs(ranks[0]["norm"] - float(bucket.norm())) <= 1e-5 * float(bucket.norm())
    # HIP's clip + Adam on its own bucket == torch's
    ref_own = _adam_update(w0, bucket)
    e_own = rel_l2(hip_w, ref_own)
    # vs Adam on the fp64 oracle gradient: elementwise, except at noise-level gradients
    ref64 = _adam_update(w0, g64)
    w0f = torch.cat([w.double().reshape(-1) for w in w0])
    du_hip, du_64 = hip_w - w0f, ref64 - w0f
    bad = (du_hip - du_64).abs() > 1e-2 * 3e-5
    bad32 = ((_adam_update(w0, g32) - w0f) - du_64).abs() > 1e-2 * 3e-5  # the fp32 oracle's own disagreements
    rms = float(g64.pow(2).mean().sqrt())
    noisy = g64.abs() <= 1e-3 * rms
    print(f"\n[config D] Adam on own bucket rel {e_own:.2e}; vs fp64-oracle Adam: {int(bad.sum())} of {bad.numel()} "
          f"updates differ (fp32 oracle: {int(bad32.sum())}), all at |g| <= 1e-3 rms: "
          f"{bool((~noisy[bad]).sum() == 0)}; weights rel {rel_l2(hip_w, ref64):.2e}")
    assert e_own <= 1e-6
    assert int((bad & ~noisy).sum()) == 0
    # no more sign disagreements than the fp32 oracle's own (4289 vs 4286 measured, gpurun_out r04c/r04d logs)
    assert int(bad.sum()) <= 1.01 * int(bad32.sum()) + 1


def test_config_d_next_forward(ranks, oracle32):
    from test_gpu_ptv3 import rel_l2
    _, names, g32 = oracle32
    sd = {k: v.clone() for k, v in _model().state_dict().items()}
    upd = _adam_update([sd[k] for k in names], g32)
    off = 0
    for k in names:
        n = sd[k].numel()
        sd[k] = upd[off:off + n].view_as(sd[k]).float()
        off += n
    gs, counts = _batch(ACCUM)
    masks = _cat_masks([c["next_masks"] for c in ranks])
    with torch.no_grad():
        rp = _oracle_forward(sd, gs, counts, PERMS[ACCUM], masks, None, torch.float32)
    n = sum(counts)
    in_packed = torch.cat([gs[f].reshape(n, -1) for f in FEATS], 1)
    hip = torch.cat([torch.from_numpy(c["next_packed"]) for c in ranks])
    err = rel_l2(hip - in_packed, rp - in_packed)
    print(f"\n[config D] next train forward on the updated weights: residual rel L2 {err:.2e}")
    assert err < 1e-5
