"""Golden vectors for the point-downsampling experiments from the reference's own
`models/pcd_downsampling_methods.py` (it needs only torch + sklearn, both importable here: no stubs).  Run in
the build container only (/root/reference does not exist on the GPU box); writes tests/golden/downsample.npz
(inputs and outputs only)."""
import importlib.util
import os
import sys

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
    from splatformer_amd.scenes import make_scene
    spec = importlib.util.spec_from_file_location("pcd_ds", os.path.join(REF, "models", "pcd_downsampling_methods.py"))
    ds = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ds)
    s = make_scene(3000, 1, seed=21)
    pts = s["means"].float().contiguous()
    g = torch.Generator().manual_seed(4)
    feat = torch.randn(pts.shape[0], 23, generator=g)
    grid = torch.floor(pts * 384).int()
    out = {"points": pts.numpy(), "feat": feat.numpy(), "grid": grid.numpy()}
    # voxel
    vp, vf, vg = ds.voxel_downsample(pts, feat, grid, 0.02)
    logits = torch.randn(vp.shape[0], 5, generator=g)
    out.update(voxel_size=np.float64(0.02), vox_points=vp.numpy(), vox_feat=vf.numpy(), vox_grid=vg.numpy(),
               vox_logits=logits.numpy(),
               vox_mapped=ds.voxel_downsample_map_logits_to_original(pts, vp, logits, 0.02).numpy())
    # random + 1-NN map back
    torch.manual_seed(123)
    rp, rf, rg, ridx = ds.random_downsample(pts, feat, grid, 0.5)
    rlog = torch.randn(rp.shape[0], 5, generator=g)
    out.update(rnd_seed=np.int64(123), rnd_ratio=np.float64(0.5), rnd_points=rp.numpy(), rnd_feat=rf.numpy(),
               rnd_grid=rg.numpy(), rnd_idx=ridx.numpy(), rnd_logits=rlog.numpy(),
               rnd_mapped=ds.knn_map_back(rlog, rp, pts).numpy())
    # furthest point sampling + 1-NN assignment
    torch.manual_seed(7)
    cidx = ds.furthest_point_sampling(pts, 300)
    torch.manual_seed(7)
    fp_, ff, fg, fa = ds.fps_knn_downsample(pts, feat, grid, 0.1)
    out.update(fps_seed=np.int64(7), fps_ratio=np.float64(0.1), fps_centroids=cidx.numpy(), fps_points=fp_.numpy(),
               fps_feat=ff.numpy(), fps_grid=fg.numpy(), fps_assign=fa.numpy())
    np.savez_compressed(os.path.join(OUT, "downsample.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
