"""Config D semantics on one GPU: two ranks (gloo, both on cuda:0), one scene each, SyncBatchNorm statistics
and the DDP gradient-bucket average, vs the oracle's single forward over the 2-scene batch (whose
BatchNorms see both scenes, exactly SyncBatchNorm's statistics) -- PTv3 backbone, train mode.

DDP averages the per-rank qkv gradients: (g0 + g1) / 2 must equal half the gradient of the batch loss
sum_r <feat_r, dfeat_r>.  Bar: as close to the fp64 oracle as the fp32 oracle (2x + 1e-5)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

PERMS = [[1, 0, 3, 2], [2, 3, 0, 1], [0, 1, 2, 3], [3, 2, 1, 0], [1, 3, 0, 2]]
SMALL = ((2500, 2200), True)       # per-rank scene sizes, unique stage-0 voxels
LARGE = ((100_000, 100_000), False)  # config D's workload: 100k Gaussians per rank, duplicate voxels kept


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scene(r, sizes=SMALL):
    from splatformer_amd.scenes import make_scene
    return make_scene(sizes[0][r], 1, seed=40 + r, unique_voxels=sizes[1])


def _worker(rank, world, port, q, sizes=SMALL):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    try:
        import torch.distributed as tdist
        from oracle import ptv3_ref
        from splatformer_amd import dist, ptv3_train as pt
        from test_gpu_ptv3 import _model
        from test_gpu_train import RecordingMasks
        tdist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        model = _model(41).to(dev)
        for name, p in model.named_parameters():
            p.requires_grad_("attn.qkv" in name)
        params = [p for p in model.parameters() if p.requires_grad]
        flat = torch.zeros(sum(p.numel() for p in params), device=dev)
        off = 0
        for p in params:
            p.grad = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        s = _scene(rank, sizes)
        n = s["means"].shape[0]
        data = ptv3_ref.batchify(s)
        dd = {k: (v.to(dev) if isinstance(v, torch.Tensor) else v) for k, v in data.items()}
        dd["offset"] = [n]
        masks = RecordingMasks(100 + rank)
        point, tape = pt.backbone_forward(model.backbone.backbone, dd, masks, perms=PERMS,
                                          group=tdist.group.WORLD)
        dfeat = torch.randn(point.feat.shape, generator=torch.Generator().manual_seed(7 + rank))
        pt.backbone_backward(tape, dfeat.to(dev))
        dist.allreduce_mean_(flat)
        torch.cuda.synchronize()
        # numpy payloads: pickled by value (tensor payloads would be shared-memory fds that die with the rank)
        q.put((rank, flat.cpu().numpy(), {k: v.numpy() for k, v in masks.masks.items()}, dfeat.numpy(),
               point.feat.cpu().numpy()))
        tdist.barrier()
    finally:
        if torch.distributed.is_initialized():
            torch.distributed.destroy_process_group()


def _run_ranks(sizes, world=2):
    """Both ranks' (averaged bucket, DropPath masks, dfeat, features), HIP side."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, sizes)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=600) for _ in range(world)), key=lambda t: t[0])
    res = [(r, torch.from_numpy(f), {k: torch.from_numpy(v) for k, v in m.items()}, torch.from_numpy(d),
            torch.from_numpy(x)) for r, f, m, d, x in res]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert torch.equal(res[0][1], res[1][1])  # every rank holds the same averaged bucket
    return res


def _oracle_batch(res, sizes, dtype, world=2):
    """The oracle's single train forward over the ranks' scenes as one batch (its BatchNorms see every scene:
    SyncBatchNorm's statistics) + autograd of sum_r <feat_r, dfeat_r>; -> (qkv grads / world, features)."""
    from oracle import ptv3_ref
    from test_gpu_ptv3 import _model
    model = _model(41)
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    names = [k for k, p in model.named_parameters() if "attn.qkv" in k]
    datas = [ptv3_ref.batchify(_scene(r, sizes)) for r in range(world)]
    counts = [d["feat"].shape[0] for d in datas]
    batch = dict(coord=torch.cat([d["coord"] for d in datas]), feat=torch.cat([d["feat"] for d in datas]),
                 grid_coord=torch.cat([d["grid_coord"] for d in datas]),
                 offset=torch.tensor([counts[0], counts[0] + counts[1]]))
    masks = {k: torch.cat([res[0][2][k], res[1][2][k]]) for k in res[0][2]}
    dfeat = torch.cat([res[0][3], res[1][3]])
    prev = torch.get_default_dtype()
    torch.set_default_dtype(dtype)
    try:
        sdd = {k: (v.to(dtype) if v.is_floating_point() else v).clone() for k, v in sd.items()}
        for k in names:
            sdd[k].requires_grad_()
        dat = {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in batch.items()}
        pnt = ptv3_ref.ptv3_forward(sdd, ptv3_ref.PTv3Config(), dat, PERMS, prefix="backbone.backbone.", train=True,
                                    masks={k: m.to(dtype) for k, m in masks.items()})
        (pnt.feat * dfeat.to(dtype)).sum().backward()
    finally:
        torch.set_default_dtype(prev)
    return torch.cat([sdd[k].grad.double().reshape(-1) for k in names]) / world, pnt.feat.detach()


def test_two_rank_syncbn_ddp_grads(device):
    from test_gpu_ptv3 import rel_l2
    res = _run_ranks(SMALL)
    flat_hip = res[0][1].double()
    g32, f32 = _oracle_batch(res, SMALL, torch.float32)
    assert rel_l2(torch.cat([res[0][4], res[1][4]]), f32) < 1e-5  # per-rank features == batch features
    g64, _ = _oracle_batch(res, SMALL, torch.float64)
    e_hip, e_ref = rel_l2(flat_hip, g64), rel_l2(g32, g64)
    print(f"\n[ddp x2] HIP {e_hip:.2e} fp32 oracle {e_ref:.2e} (to fp64)")
    assert e_hip <= 2.0 * e_ref + 1e-5


# ---- config D's workload: 100k Gaussians per rank -----------------------------------------
@pytest.fixture(scope="module")
def ddp_large(device):
    return _run_ranks(LARGE)


@pytest.fixture(scope="module")
def ddp_large_oracle32(ddp_large):
    return _oracle_batch(ddp_large, LARGE, torch.float32)


@pytest.mark.timeout(900)
def test_two_rank_syncbn_ddp_100k_forward(ddp_large, ddp_large_oracle32):
    from test_gpu_ptv3 import rel_l2
    _, f32 = ddp_large_oracle32
    err = rel_l2(torch.cat([ddp_large[0][4], ddp_large[1][4]]), f32)
    print(f"\n[ddp x2, 100k/rank] train features rel L2 {err:.2e}")
    assert err < 1e-5


@pytest.mark.timeout(900)
def test_two_rank_syncbn_ddp_100k_grads(ddp_large, ddp_large_oracle32):
    from test_gpu_ptv3 import rel_l2
    g32, _ = ddp_large_oracle32
    g64, _ = _oracle_batch(ddp_large, LARGE, torch.float64)
    e_hip, e_ref = rel_l2(ddp_large[0][1].double(), g64), rel_l2(g32, g64)
    print(f"\n[ddp x2, 100k/rank] HIP {e_hip:.2e} fp32 oracle {e_ref:.2e} (to fp64)")
    assert e_hip <= 2.0 * e_ref + 1e-5
