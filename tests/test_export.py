"""Viewer export (splatformer_amd/export.py) against golden vectors captured from the reference's own
utils/gs_utils.py export_ply_forviewer / prepare_viewer (tests/golden/make_golden.py part 5).  CPU only."""
import json
import os

import numpy as np
import torch

from splatformer_amd import export

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "export.npz")


def test_ply_vertices_match_reference(tmp_path):
    d = np.load(GOLD)
    for deg in (1, 0):
        gs = {k[len(f"deg{deg}_in_"):]: torch.from_numpy(d[k]) for k in d.files if k.startswith(f"deg{deg}_in_")}
        want = d[f"deg{deg}_vertices"]
        el = export.ply_attributes(gs)
        assert el.dtype.names == want.dtype.names
        assert el.tobytes() == np.ascontiguousarray(want).astype(el.dtype).tobytes()
        path = os.path.join(str(tmp_path), "out", f"deg{deg}.ply")
        export.export_ply_forviewer(gs, path)
        back = export.read_ply(path)
        assert back.dtype.names == want.dtype.names and back.tobytes() == el.tobytes()
        with open(path, "rb") as f:
            head = f.read(64).split(b"\n")
        assert head[0] == b"ply" and head[1] == b"format binary_little_endian 1.0"


def test_viewer_cameras_match_reference(tmp_path):
    d = np.load(GOLD)
    fx, fy, w, h = d["cam_intr"]
    cams = {"camera_to_worlds": torch.from_numpy(d["cam_c2w"]), "fx": torch.tensor(float(fx)),
            "fy": torch.tensor(float(fy)), "width": torch.tensor(int(w)), "height": torch.tensor(int(h))}
    export.prepare_viewer(cams, str(tmp_path), 1)
    got = json.load(open(os.path.join(str(tmp_path), "cameras.json")))
    want = json.loads(str(d["cameras_json"]))
    assert got == want
    assert open(os.path.join(str(tmp_path), "cfg_args")).read() == str(d["cfg_args"])
