"""Debug: culled vs full eval render on the test_batched_views scene; quad kernel on the full list."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splatformer_amd import _lib, gs_render
from splatformer_amd._lib import call, ptr, stream
from splatformer_amd.scenes import make_cameras, make_scene, to_device

_lib.load()
dev = torch.device("cuda", 0)
s = to_device(make_scene(20000, 1, seed=12), dev)
cams = to_device(make_cameras(160, 120, n_views=5), dev)
with torch.no_grad():
    gs_render.RENDER_CULL = True
    rc, ac, mc = gs_render.render_views_meta(s, cams)
    gs_render.RENDER_CULL = False
    rf, af, mf = gs_render.render_views_meta(s, cams)
torch.cuda.synchronize()
print("isect culled", mc["isect_sorted"].numel(), "full", mf["isect_sorted"].numel())
for v in range(5):
    d = (rc[v] - rf[v]).abs()
    nz = (d.sum(-1) > 0).nonzero()
    print("view", v, "rgb diff pixels", nz.shape[0], "max", float(d.max()), "first", nz[:8].tolist())
# quad kernel over the FULL list
V, H, W = 5, 120, 160
tx, ty = 10, 8
rec = torch.empty(V * 20000, 12, device=dev)
call("sfx_pack_raster_records", V * 20000, ptr(mf["xys"]), ptr(mf["conics"]), ptr(mf["rgbs"]), ptr(mf["opacities"]),
     ptr(rec), stream())
bg = cams["background_color"].float().contiguous()
outs = {}
for k in ("sfx_rasterize_fwd_views_packed", "sfx_rasterize_fwd_views_quad"):
    o = torch.empty(V, H, W, 3, device=dev); a = torch.empty(V, H, W, device=dev)
    fT = torch.empty(V, H, W, device=dev); fi = torch.empty(V, H, W, device=dev, dtype=torch.int32)
    call(k, V, tx, ty, 16, H, W, ptr(mf["gids_sorted"]), ptr(mf["tile_bins"]), ptr(rec), ptr(bg), 1, ptr(fT), ptr(fi),
         ptr(o), ptr(a), stream())
    outs[k] = (o, a, fT, fi)
torch.cuda.synchronize()
p, q = outs["sfx_rasterize_fwd_views_packed"], outs["sfx_rasterize_fwd_views_quad"]
for i, nm in enumerate(["rgb", "alpha", "T", "idx"]):
    d = (p[i].double() - q[i].double()).abs()
    print("full list, packed vs quad", nm, "n diff", int((d > 0).sum()), "max", float(d.max()))
    if int((d > 0).sum()):
        print("  first", (d.reshape(V, H, W, -1).sum(-1) > 0).nonzero()[:8].tolist())
