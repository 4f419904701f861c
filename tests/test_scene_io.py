"""Scene I/O (splatformer_amd/scene_io.py) against golden vectors captured from the reference's own
dataset/GS.py loaders (tests/golden/make_golden.py part 3): bit-exact Gaussian parameters after the NaN /
outlier / truncation / MinMax / inf-range filters, normalised camera poses, the OOD test split and RGBA
compositing.  CPU only."""
import os
import pickle

import numpy as np
import pytest
import torch

from splatformer_amd import scene_io

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "scene_io.npz")
FEATS = ["means", "scales", "opacities", "quats", "features_dc", "features_rest"]


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


def _write_scene(root, d, extra_ckpt=False):
    ns = os.path.join(root, "scene0", "splatfacto")
    os.makedirs(os.path.join(ns, "nerfstudio_models"))
    ck = {"_model.gauss_params." + k: torch.from_numpy(d["in_" + k]) for k in FEATS}
    ck["step"] = 29999
    torch.save(ck, os.path.join(ns, "nerfstudio_models", "step-000029999.ckpt"))
    if extra_ckpt:  # an older checkpoint: the loader must take the last step
        torch.save({"step": 100}, os.path.join(ns, "nerfstudio_models", "step-000000100.ckpt"))
    meta = {k[len("in_meta_"):]: torch.from_numpy(np.array(d[k])) for k in d.files if k.startswith("in_meta_")}
    with open(os.path.join(ns, "camera_for-3d-denoise.pkl"), "wb") as f:
        pickle.dump(meta, f)
    cm = os.path.join(root, "colmap", "scene0")
    os.makedirs(os.path.join(cm, "images"))
    names = [f"frame_{i:03d}.png" for i in range(5)]
    names += [f"elevation{e}_azimuth{a}.png" for e in (30, 70, 80, 90) for a in (0, 120, 240)]
    for nm in names:
        open(os.path.join(cm, "images", nm), "wb").close()
    return ns, cm


@pytest.mark.parametrize("ndevs", [0, 3])
def test_load_scene_matches_reference(tmp_path, gold, ndevs):
    ns, cm = _write_scene(str(tmp_path), gold, extra_ckpt=True)
    sc = scene_io.load_scene(ns, cm, FEATS, max_gs_num=1000, remove_outlier_ndevs=ndevs)
    p = f"nd{ndevs}_"
    for k in FEATS:
        np.testing.assert_array_equal(sc["gs_params"][k].numpy(), gold[p + k], err_msg=k)
    np.testing.assert_array_equal(sc["meta"]["test_camera_to_worlds"].numpy(), gold[p + "test_c2w"])
    np.testing.assert_array_equal(sc["meta"]["train_camera_to_worlds"].numpy(), gold[p + "train_c2w"])
    assert [os.path.basename(x) for x in sc["test_imgs_path"]] == list(gold[p + "test_names"])
    assert [os.path.basename(x) for x in sc["train_imgs_path"]] == list(gold[p + "train_names"])
    cams = sc["cameras"]
    assert cams["camera_to_worlds"].shape == (9, 3, 4) and float(cams["fx"]) == float(gold["in_meta_fx"])
    # the filters did their work: no NaN / inf, means inside the unit cube, at most max_gs_num points
    m = sc["gs_params"]["means"]
    assert m.shape[0] <= 1000 and bool(((m >= 0) & (m <= 1)).all())
    assert all(torch.isfinite(v).all() for v in sc["gs_params"].values())


def test_read_image_rgba_composite(tmp_path, gold):
    from PIL import Image
    path = os.path.join(str(tmp_path), "rgba.png")
    Image.fromarray(gold["in_rgba"], "RGBA").save(path)
    out = scene_io.read_image(path, torch.from_numpy(gold["rgba_bg"]))
    np.testing.assert_array_equal(out.numpy(), gold["rgba_out"])


def test_camera_pickle_is_restricted(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))
    path = os.path.join(str(tmp_path), "cam.pkl")
    with open(path, "wb") as f:
        pickle.dump({"fx": Evil()}, f)
    with pytest.raises(pickle.UnpicklingError):
        scene_io.load_camera_pickle(path)


def test_scaler_roundtrip_and_outliers():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(500, 3, generator=g) * torch.tensor([3.0, 1.0, 0.2])
    s = scene_io.MinMaxScaler()
    y = s.fit_transform(x)
    assert float(y.min()) >= -1e-6 and float(y.max()) <= 1 + 1e-6  # (rounding: the loader filters [0,1])
    torch.testing.assert_close(s.inverse_transform(y), x, rtol=1e-5, atol=1e-5)
    x[3] = 100.0
    _, mask = scene_io.remove_outliers(x, 3)
    assert not bool(mask[3]) and int(mask.sum()) >= 480
