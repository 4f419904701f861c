"""Per-output mismatch counts of the HIP projection vs the oracle (same float inputs), with the first mismatching
Gaussian's inputs dumped for a host-side emulation."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from oracle import gsplat_ref, render_ref
from splatformer_amd import gsplat_compat, _lib
from splatformer_amd.scenes import make_cameras, make_scene
_lib.load()
dev = torch.device("cuda:0")
s = make_scene(5000, 1, 0)
cams = make_cameras(160, 120, n_views=9)
a = render_ref.glue_args(s, cams["camera_to_worlds"][0])
args = (a["means"], a["scales"], 1.0, a["quats"], a["viewmat"], cams["fx"], cams["fy"], cams["cx"], cams["cy"], 120, 160, 16)
ref = gsplat_ref.project_gaussians(*args)
out = gsplat_compat.project_gaussians(*[x.to(dev) if isinstance(x, torch.Tensor) else x for x in args])
names = ["xys", "depths", "radii", "conics", "comp", "num_tiles_hit", "cov3d"]
res = {}
for nm, r, o in zip(names, ref, out):
    o = o.cpu()
    res[nm] = int((r != o).sum())
print(json.dumps(res))
bad = torch.nonzero((ref[6] != out[6].cpu()).any(-1)).flatten()
if bad.numel():
    i = int(bad[0])
    np.set_printoptions(precision=10)
    print("first cov3d mismatch", i, "oracle", ref[6][i].numpy().tolist(), "hip", out[6][i].cpu().numpy().tolist())
    print("inputs", a["means"][i].numpy().tolist(), a["scales"][i].numpy().tolist(), a["quats"][i].numpy().tolist())
    print("bits scales", a["scales"][i].numpy().view(np.uint32).tolist(), "quats", a["quats"][i].numpy().view(np.uint32).tolist())
