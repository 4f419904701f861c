"""Debug helper: trace the refiner backward of two identical runs and report the first diverging tensor."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from splatformer_amd import ptv3_train as pt  # noqa: E402
from splatformer_amd import train as strain  # noqa: E402
from splatformer_amd.scenes import make_scene, to_device  # noqa: E402
from test_gpu_ptv3 import _model, rel_l2  # noqa: E402
from test_gpu_train import RecordingMasks  # noqa: E402

dev = torch.device("cuda")


def run(bk, n, use_masks, seed_m):
    model = _model(21, **bk).to(dev)
    for name, p in model.named_parameters():
        p.requires_grad_("attn.qkv" in name)
        p.grad = torch.zeros_like(p) if p.requires_grad else None
    s = make_scene(n, 1, seed=n + 1, unique_voxels=True)
    masks = RecordingMasks(seed_m) if use_masks else (lambda name, n, p, device=None: None)
    torch.manual_seed(5)
    pt._TRACE = []
    packed, tape = strain.refine_train(model, to_device(s, dev), masks)
    d = torch.randn(packed.shape, generator=torch.Generator().manual_seed(9))
    strain.refine_backward(model, tape, d.to(dev))
    torch.cuda.synchronize()
    tr = [(k, v.cpu()) for k, v in pt._TRACE]
    pt._TRACE = None
    return tr


bk1 = dict(enc_depths=(1, 1, 1, 1, 1), dec_depths=(1, 1, 1, 1))
run(bk1, 2000, False, 0)
a = run(bk1, 2000, True, 2014)
b = run(bk1, 2000, True, 2014)
shown = 0
for (ka, va), (kb, vb) in zip(a, b):
    e = rel_l2(va, vb)
    if e > 1e-5:
        print(f"{ka}: {e:.2e}", flush=True)
        shown += 1
        if shown > 25:
            break
print("compared", len(a), len(b))
