"""Config D's per-GPU step at its own workload: train-on-objaverse gpux8-accum4 runs, on every
rank, `accumulate_step` = 4 micro-steps of one 100k-Gaussian SH1 scene with 4 training views at 800x800 (reference
train.py:227-303: loss / accumulate_step at :286, the gradients summed in place, then clip_grad_norm_(2.0) and
Adam(lr 3e-5, eps 1e-15) on attn.qkv, utils/optimizers.py:46-52, configs/train/default.gin).  One GPU here: the
8-rank DDP all-reduce of the bucket is the driver's multi-GPU run (its semantics are tests/test_gpu_config_d.py's,
2 ranks at small sizes); this file runs the per-GPU work at full size, with no oracle (sizes the CPU oracle would
need minutes for):

* the accumulated bucket == the sum of the four micro-steps' gradients taken individually (each micro-step run
  alone from a zero bucket, same scene, views, order shuffles and DropPath masks): relative L2 within the run-to-run
  noise of the training step's float atomics (bar printed with the measured value);
* the bucket is still accumulating after micro-steps 1-3 (no optimiser step, no reset) and is zeroed by the step;
* the optimiser step: HIP's clip + Adam == torch.nn.utils.clip_grad_norm_ + torch.optim.Adam applied to the same
  bucket (fp64 copies), relative L2 of the updated weights <= 1e-6, and the norm HIP clipped with == the bucket's.
"""
import pytest
import torch

from splatformer_amd import gs_render
from splatformer_amd import train as strain
from splatformer_amd.scenes import make_cameras, make_scene, to_device
from test_gpu_ptv3 import rel_l2
from test_gpu_train import RecordingMasks

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

N, RES, VIEWS, ACCUM = 100_000, 800, 4, 4
PERMS = [[[1, 0, 3, 2], [2, 3, 0, 1], [0, 1, 2, 3], [3, 2, 1, 0], [1, 3, 0, 2]],
         [[0, 1, 2, 3], [1, 2, 3, 0], [3, 0, 2, 1], [2, 1, 0, 3], [0, 3, 1, 2]],
         [[3, 2, 1, 0], [0, 1, 2, 3], [1, 0, 3, 2], [2, 0, 3, 1], [3, 1, 2, 0]],
         [[2, 3, 0, 1], [3, 0, 1, 2], [0, 2, 1, 3], [1, 3, 2, 0], [2, 1, 3, 0]]]


class ReplayMasks:
    """DropPath masks recorded by a RecordingMasks run, handed out again by name (the same draws)."""

    def __init__(self, masks, device):
        self.masks = {k: v.to(device) for k, v in masks.items()}

    def __call__(self, name, n, p, device=None):
        return self.masks.get(name) if p > 0 else None


def _model(device):
    from splatformer_amd.feature_predictor import FeaturePredictor
    torch.manual_seed(0)
    return FeaturePredictor(sh_degree=1, zeroinit=False).to(device)


@pytest.fixture(scope="module")
def run_d(device):
    cams = to_device(make_cameras(RES, RES, n_views=VIEWS), device)
    scenes = [to_device(make_scene(N, 1, seed=40 + i), device) for i in range(ACCUM)]
    with torch.no_grad():
        gts = [[g.clone() for g in gs_render.rasterize_gaussians_to_multiimgs(s, cams)[0]] for s in scenes]
    model = _model(device)
    tr = strain.Trainer(model, accumulate_step=ACCUM)
    assert (tr.lr, tr.eps, tr.clip) == (3e-5, 1e-15, 2.0)
    names = [k for k, p in model.named_parameters() if p.requires_grad]
    w0 = {k: p.detach().clone() for k, p in model.named_parameters() if p.requires_grad}
    rec, still = [], []
    for i in range(ACCUM):
        masks = RecordingMasks(700 + i)
        tr.micro_step([scenes[i]], [cams], [gts[i]], masks=masks, perms=PERMS[i])
        rec.append({k: v.clone() for k, v in masks.masks.items()})
        still.append(float(tr.flat_grad.abs().max()))
    bucket = tr.flat_grad.detach().clone()
    orig_clip = strain.tops.grad_clip_coef
    seen = {}

    def clip(grads, max_norm):
        coef, norm = orig_clip(grads, max_norm)
        seen["norm"] = norm
        return coef, norm
    strain.tops.grad_clip_coef = clip
    try:
        tr.optimizer_step()
    finally:
        strain.tops.grad_clip_coef = orig_clip
    torch.cuda.synchronize()
    upd = {k: p.detach().clone() for k, p in model.named_parameters() if p.requires_grad}
    zeroed = float(tr.flat_grad.abs().max())

    # each micro-step alone, from a zero bucket, on the pre-step weights (replayed masks and order shuffles)
    def alone(i):
        m = _model(device)
        t = strain.Trainer(m, accumulate_step=ACCUM)
        t.micro_step([scenes[i]], [cams], [gts[i]], masks=ReplayMasks(rec[i], device), perms=PERMS[i])
        torch.cuda.synchronize()
        return t.flat_grad.detach().clone()
    singles = [alone(i) for i in range(ACCUM)]
    again = alone(0)  # run-to-run noise of one micro-step (float atomics of the training kernels)
    return dict(bucket=bucket.cpu(), singles=[s.cpu() for s in singles], again=again.cpu(), still=still,
                zeroed=zeroed, w0=[w0[k].cpu() for k in names], upd=[upd[k].cpu() for k in names],
                norm=float(seen["norm"]), step_count=tr.step_count)


def test_config_d_full_accumulates(run_d):
    assert all(v > 0 for v in run_d["still"]) and run_d["step_count"] == 1 and run_d["zeroed"] == 0.0
    b = run_d["bucket"].double()
    s = torch.stack(run_d["singles"]).double().sum(0)
    e = rel_l2(b, s)
    noise = rel_l2(run_d["again"].double(), run_d["singles"][0].double())
    bar = max(8.0 * noise, 1e-5)
    print(f"\n[config D full, 100k x 4 views 800^2 x accum 4] bucket vs sum of the micro-steps taken alone: rel L2 "
          f"{e:.2e} (one micro-step run twice: {noise:.2e}; bar {bar:.1e})")
    assert e <= bar


def test_config_d_full_optimizer_step(run_d):
    b = run_d["bucket"].double()
    assert abs(run_d["norm"] - float(b.norm())) <= 1e-5 * float(b.norm())
    ps = [torch.nn.Parameter(w.clone().double()) for w in run_d["w0"]]
    off = 0
    for p in ps:
        p.grad = b[off:off + p.numel()].view_as(p).clone()
        off += p.numel()
    torch.nn.utils.clip_grad_norm_(ps, 2.0)
    torch.optim.Adam(ps, lr=3e-5, eps=1e-15).step()
    ref = torch.cat([p.detach().reshape(-1) for p in ps])
    hip = torch.cat([u.double().reshape(-1) for u in run_d["upd"]])
    w0 = torch.cat([w.double().reshape(-1) for w in run_d["w0"]])
    e = rel_l2(hip, ref)
    e_delta = rel_l2(hip - w0, ref - w0)
    print(f"\n[config D full] HIP clip + Adam vs torch.optim.Adam on the same bucket: weights rel {e:.2e}, "
          f"updates rel {e_delta:.2e}")
    assert e <= 1e-6 and e_delta <= 1e-4
