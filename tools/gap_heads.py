"""Where the gap before the heads comes from: host time between the backbone returning and the heads launch vs
the GPU time between the two events.  usage: python tools/gap_heads.py"""
import os, sys, time, statistics
import torch
sys.path.insert(0, os.getcwd())
from splatformer_amd import _lib, ptv3_ops as ops
from splatformer_amd import feature_predictor as fpm
from splatformer_amd.feature_predictor import FeaturePredictor
from splatformer_amd.gs_render import rasterize_gaussians_to_multiimgs
from splatformer_amd.scenes import make_cameras, make_scene, to_device
dev = torch.device("cuda", 0)
_lib.load()
torch.manual_seed(0)
model = FeaturePredictor(sh_degree=1, zeroinit=False).eval().to(dev)
scene = to_device(make_scene(100_000, sh_degree=1, seed=0), dev)
cams = to_device(make_cameras(800, 800, n_views=9), dev)
T = {}
orig_bb = model.backbone.forward
def bb(*a, **k):
    r = orig_bb(*a, **k)
    e = torch.cuda.Event(enable_timing=True); e.record(); T['bb_end_ev'] = e; T['bb_end_h'] = time.perf_counter()
    return r
model.backbone.forward = bb
orig_heads = ops.heads
def hd(*a, **k):
    T['heads_h'] = time.perf_counter()
    e = torch.cuda.Event(enable_timing=True); e.record(); T['heads_ev'] = e
    r = orig_heads(*a, **k)
    e2 = torch.cuda.Event(enable_timing=True); e2.record(); T['heads_end_ev'] = e2
    return r
ops.heads = hd
res = []
def step():
    t0 = time.perf_counter()
    out = model([scene], [0])[0]
    t1 = time.perf_counter()
    r = rasterize_gaussians_to_multiimgs(out, cams)[0]
    return t0, t1
for _ in range(3): step()
torch.cuda.synchronize()
for _ in range(10):
    t0, t1 = step()
    torch.cuda.synchronize()
    res.append((T['heads_h'] - T['bb_end_h'], T['bb_end_ev'].elapsed_time(T['heads_ev']) * 1e3, T['heads_ev'].elapsed_time(T['heads_end_ev']) * 1e3, (t1 - t0) * 1e3))
for r in res: print("host bb_end->heads %.1f us | gpu bb_end->heads %.1f us | heads %.1f us | model() host %.2f ms" % r)
