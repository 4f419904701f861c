"""Count integer mismatches (radii, num_tiles_hit) of the HIP projection vs the CPU oracle on the config-B
scene (100k Gaussians SH1, 9 views 800x800), identical float inputs (oracle glue on the CPU)."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from oracle import gsplat_ref, render_ref
from splatformer_amd import gsplat_compat, _lib
from splatformer_amd.scenes import make_cameras, make_scene
_lib.load()
dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
s = make_scene(n, 1, 0)
cams = make_cameras(800, 800, n_views=9)
res = []
for v in range(9):
    a = render_ref.glue_args(s, cams["camera_to_worlds"][v])
    args = (a["means"], a["scales"], 1.0, a["quats"], a["viewmat"], cams["fx"], cams["fy"], cams["cx"], cams["cy"], 800, 800, 16)
    ref = gsplat_ref.project_gaussians(*args)
    out = gsplat_compat.project_gaussians(*[x.to(dev) if isinstance(x, torch.Tensor) else x for x in args])
    res.append({"view": v, "radii": int((ref[2] != out[2].cpu()).sum()), "tiles": int((ref[5] != out[5].cpu()).sum()),
                "xys_maxdiff": float((ref[0] - out[0].cpu()).abs().max())})
print(json.dumps({"n": n, "per_view": res, "radii_total": sum(r["radii"] for r in res),
                  "tiles_total": sum(r["tiles"] for r in res)}))
