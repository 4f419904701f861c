"""Viewer export of refined Gaussians (reference utils/gs_utils.py:119-261).

* `export_ply_forviewer(gs, filename)` -- gs_utils.py:163-209 + write_ply_v2 :211-261: the Inria 3DGS vertex
  layout (x y z nx ny nz f_dc_* f_rest_* opacity scale_* rot_*, all float32; f_rest in the Inria order =
  features_rest transposed to [N, 3, K-1]; SH-degree-0 scenes store RGB2SH(sigmoid(features_dc))), written as
  the binary little-endian PLY that plyfile's `PlyData([el]).write` produces -- without the plyfile package
  (absent here), by a direct numpy writer.
* `prepare_viewer(cameras, dirname, sh_degree)` -- gs_utils.py:119-161: `cfg_args` and `cameras.json` for the
  SIBR / Inria viewer (OpenGL c2w -> COLMAP flip, world-to-camera inversion, FoV from focal lengths).
* `read_ply(filename)` -- the inverse of the writer (structured numpy array), for tests and tooling.

Host-side file formats (numpy on CPU): the refined record is copied off the device once per export.  Pinned
by golden vectors captured from the reference's own export code (tests/golden/make_golden.py part 5).
"""
from __future__ import annotations

import json
import math
import os
from argparse import Namespace
from collections import OrderedDict
from typing import Dict

import numpy as np
import torch

C0 = 0.28209479177387814  # gs_utils.py:14


def rgb2sh(rgb):
    return (rgb - 0.5) / C0


def ply_attributes(gs: Dict[str, torch.Tensor]) -> np.ndarray:
    """The structured vertex array of export_ply_forviewer / write_ply_v2 (gs_utils.py:163-259)."""
    with torch.no_grad():
        pos = gs["means"].detach().float().cpu().numpy()
        n = pos.shape[0]
        cols = OrderedDict()
        cols["x"], cols["y"], cols["z"] = pos[:, 0], pos[:, 1], pos[:, 2]
        cols["nx"] = cols["ny"] = cols["nz"] = np.zeros(n, dtype=np.float32)
        rest = gs.get("features_rest")
        if rest is not None and rest.shape[1] != 0:
            dc = gs["features_dc"].detach().float().contiguous().cpu().numpy()
            sh_rest = rest.detach().float().transpose(1, 2).contiguous().cpu().numpy().reshape(n, -1)
        else:  # SH degree 0: the stored dc is a colour logit
            dc = rgb2sh(torch.sigmoid(gs["features_dc"].detach().float())).cpu().numpy()
            sh_rest = np.zeros((n, 0), dtype=np.float32)
        for i in range(dc.shape[1]):
            cols[f"f_dc_{i}"] = dc[:, i]
        for i in range(sh_rest.shape[1]):
            cols[f"f_rest_{i}"] = sh_rest[:, i]
        cols["opacity"] = gs["opacities"].detach().float().cpu().numpy().reshape(n)
        sc = gs["scales"].detach().float().cpu().numpy()
        for i in range(3):
            cols[f"scale_{i}"] = sc[:, i]
        q = gs["quats"].detach().float().cpu().numpy()
        for i in range(4):
            cols[f"rot_{i}"] = q[:, i]
    el = np.empty(n, dtype=[(k, "<f4") for k in cols])
    for k, v in cols.items():
        el[k] = v
    return el


def write_ply(path: str, vertices: np.ndarray) -> None:
    """Binary little-endian PLY with one `vertex` element (the file plyfile writes for write_ply_v2)."""
    header = ["ply", "format binary_little_endian 1.0", f"element vertex {vertices.shape[0]}"]
    header += [f"property float {name}" for name in vertices.dtype.names]
    header.append("end_header")
    with open(path, "wb") as f:
        f.write(("\n".join(header) + "\n").encode("ascii"))
        f.write(np.ascontiguousarray(vertices).tobytes())


def read_ply(path: str) -> np.ndarray:
    """Read a PLY written by write_ply (binary little-endian float vertex properties)."""
    with open(path, "rb") as f:
        names, n = [], None
        line = f.readline().decode("ascii").strip()
        if line != "ply":
            raise ValueError(f"{path}: not a PLY file")
        while True:
            line = f.readline().decode("ascii").strip()
            if line == "end_header":
                break
            parts = line.split()
            if parts[0] == "format" and parts[1] != "binary_little_endian":
                raise ValueError(f"{path}: unsupported PLY format {parts[1]}")
            if parts[0] == "element":
                n = int(parts[2])
            elif parts[0] == "property":
                if parts[1] != "float":
                    raise ValueError(f"{path}: unsupported property type {parts[1]}")
                names.append(parts[2])
        return np.frombuffer(f.read(), dtype=[(k, "<f4") for k in names], count=n).copy()


def export_ply_forviewer(gs: Dict[str, torch.Tensor], filename: str) -> None:
    """gs_utils.py:163-209."""
    os.makedirs(os.path.dirname(filename) or ".", exist_ok=True)
    write_ply(str(filename), ply_attributes(gs))


def focal2fov(focal, pixels):
    return 2 * math.atan(pixels / (2 * focal))


def viewer_cameras(cameras) -> list:
    """gs_utils.py:125-158: the cameras.json records (OpenGL c2w -> COLMAP, world-to-camera inverse)."""
    out = []
    for i in range(len(cameras["camera_to_worlds"])):
        c2w_opengl = cameras["camera_to_worlds"][i]
        cam = {"id": i, "img_name": f"img_{i}.png", "width": _item(cameras["width"]),
               "height": _item(cameras["height"]), "fx": _item(cameras["fx"]), "fy": _item(cameras["fy"]),
               "FovX": None, "FovY": None, "position": None, "rotation": None}
        cam["FovX"] = focal2fov(cam["fx"], cam["width"])
        cam["FovY"] = focal2fov(cam["fy"], cam["height"])
        c2w = np.eye(4)
        c2w[:3, :4] = torch.as_tensor(c2w_opengl).cpu().numpy()[:3, :4]  # [3,4] (nerfstudio) or [4,4]
        c2w[:3, 1:3] *= -1
        w2c = np.linalg.inv(c2w)
        R = np.transpose(w2c[:3, :3])
        T = w2c[:3, 3]
        Rt = np.zeros((4, 4))
        Rt[:3, :3] = R.transpose()
        Rt[:3, 3] = T
        Rt[3, 3] = 1.0
        W2C = np.linalg.inv(Rt)
        cam["position"] = W2C[:3, 3].tolist()
        cam["rotation"] = [x.tolist() for x in W2C[:3, :3]]
        out.append(cam)
    return out


def _item(x):
    return x.item() if hasattr(x, "item") else x


def prepare_viewer(cameras, dirname: str, sh_degree: int) -> None:
    """gs_utils.py:119-161: cfg_args + cameras.json next to the exported point cloud."""
    os.makedirs(dirname, exist_ok=True)
    with open(os.path.join(dirname, "cfg_args"), "w") as f:
        f.write(str(Namespace(source_path="", sh_degree=sh_degree, white_background=False)))
    with open(os.path.join(dirname, "cameras.json"), "w") as f:
        json.dump(viewer_cameras(cameras), f)
