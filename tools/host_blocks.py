"""Host enqueue time vs GPU span of every Block / unpooling of the config-B refine (median of 10 steps): a
module whose host time exceeds its GPU span starves the GPU.  usage: python tools/host_blocks.py"""
import os, sys, time, statistics
import torch
sys.path.insert(0, os.getcwd())
from splatformer_amd import _lib
from splatformer_amd import ptv3
from splatformer_amd.feature_predictor import FeaturePredictor
from splatformer_amd.gs_render import rasterize_gaussians_to_multiimgs
from splatformer_amd.scenes import make_cameras, make_scene, to_device
dev = torch.device("cuda", 0)
_lib.load()
torch.manual_seed(0)
model = FeaturePredictor(sh_degree=1, zeroinit=False).eval().to(dev)
scene = to_device(make_scene(100_000, sh_degree=1, seed=0), dev)
cams = to_device(make_cameras(800, 800, n_views=9), dev)
rec = []
orig_block = ptv3.Block.run
orig_unpool = ptv3.SerializedUnpooling.run
def wrap(f, tag):
    def g(self, *a, **k):
        t0 = time.perf_counter()
        ev0 = torch.cuda.Event(enable_timing=True); ev0.record()
        r = f(self, *a, **k)
        ev1 = torch.cuda.Event(enable_timing=True); ev1.record()
        rec.append((tag, getattr(self, "channels", 0), time.perf_counter() - t0, ev0, ev1))
        return r
    return g
ptv3.Block.run = wrap(orig_block, "block")
ptv3.SerializedUnpooling.run = wrap(orig_unpool, "unpool")
def step():
    out = model([scene], [0])[0]
    return rasterize_gaussians_to_multiimgs(out, cams)[0]
for _ in range(3): step()
torch.cuda.synchronize()
rec.clear()
for _ in range(10): step()
torch.cuda.synchronize()
from collections import defaultdict
agg = defaultdict(lambda: [[], []])
per = len(rec) // 10
for i, (tag, c, ht, e0, e1) in enumerate(rec):
    key = (i % per, tag, c)
    agg[key][0].append(ht * 1e6); agg[key][1].append(e0.elapsed_time(e1) * 1e3)
for key in sorted(agg):
    h, g = agg[key]
    print(f"{key[0]:3d} {key[1]:7s} C={key[2]:4d} host {statistics.median(h):8.1f} us  gpu(span) {statistics.median(g):8.1f} us")
