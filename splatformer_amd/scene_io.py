"""Scene I/O upstream of the hot path: nerfstudio splatfacto checkpoints and the
camera pickle -> the normalised Gaussian dict + cameras the refiner / renderer consume.

Mirrors the reference's SplatfactoDataset loading (reference dataset/GS.py):
  * `load_gs_params_fromnerfstudio` (GS.py:153-204): last `nerfstudio_models/step-*.ckpt`, keys
    `_model.gauss_params.*`, NaN-row filter, optional n-sigma outlier filter, truncation to `max_gs_num`,
    `MinMaxScaler.fit_transform` of the means + `log(scale_)` shift of the log-scales, inf / out-of-[0,1]
    filter;
  * `load_images_cameras_fromnerfstudio` (GS.py:206-244): `camera_for-3d-denoise.pkl` + the test-split rules
    (elevation-70/80/90 OOD views = the last 9 test poses, or an `ood-test_split.txt` subset);
  * `load_scene` (GS.py:308-322): camera translations mapped by the same scaler;
  * `remove_outliers`, `MinMaxScaler` (utils/transform_utils.py:9-98, default arguments).
Golden vectors from the reference's own code pin these (tests/golden/make_golden.py part 3,
tests/test_scene_io.py).

Differences, all on the safe side: checkpoints load with `torch.load(weights_only=True)` and the camera
pickle through a restricted unpickler (containers, numbers, strings, numpy arrays, torch tensors only), where
the reference unpickles arbitrary objects; the checkpoint glob is sorted (the reference takes `glob()[-1]`,
whose order is filesystem-defined); a checkpoint that nests the parameters under nerfstudio's `pipeline` key
is accepted besides the flat layout the reference reads.
"""
from __future__ import annotations

import glob
import io
import os
import pickle
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
from torch import Tensor

GAUSS_PREFIX = "_model.gauss_params."
BASE_FEATURES = ("means", "scales", "opacities", "quats", "features_dc", "features_rest")


def remove_outliers(points: Tensor, n_devs: float = 3) -> Tuple[Tensor, Tensor]:
    """utils/transform_utils.py:9-42 (default branch): keep points within mean +- n_devs * std per axis."""
    mean = torch.mean(points, axis=0)
    std_dev = torch.std(points, axis=0)
    lower_bound = mean - n_devs * std_dev
    upper_bound = mean + n_devs * std_dev
    mask = torch.all((points >= lower_bound) & (points <= upper_bound), axis=1)
    return points[mask], mask


class MinMaxScaler:
    """utils/transform_utils.py:44-98 with feature_range (0, 1), preserve_ratio=True: one isotropic scale, the
    scaled bounding box centred at 0.5."""

    def __init__(self, feature_range=(0, 1)):
        self.feature_range = feature_range
        self.scale_ = None
        self.trans_ = None

    def fit_transform(self, X: Tensor) -> Tensor:
        self.data_min_ = torch.min(X, dim=0)[0]
        self.data_max_ = torch.max(X, dim=0)[0]
        self.data_range_ = self.data_max_ - self.data_min_
        lo, hi = self.feature_range
        self.center = (lo + hi) / 2
        self.scale_ = torch.min((hi - lo) / self.data_range_)
        self.min_ = lo - self.data_min_ * self.scale_
        scaled = X * self.scale_
        mid = (scaled.min(dim=0)[0] + scaled.max(dim=0)[0]) / 2
        self.trans_ = self.center - mid
        return scaled + self.trans_

    def transform(self, X: Tensor) -> Tensor:
        return X * self.scale_ + self.trans_

    def inverse_transform(self, X: Tensor) -> Tensor:
        return (X - self.trans_) / self.scale_


def _last_checkpoint(nerfstudio_dir: str) -> str:
    files = sorted(glob.glob(os.path.join(nerfstudio_dir, "nerfstudio_models", "step-*.ckpt")))
    if not files:
        raise FileNotFoundError(f"{nerfstudio_dir} has no nerfstudio_models/step-*.ckpt")
    return files[-1]


def load_gs_params_fromnerfstudio(nerfstudio_dir: str, input_features: Sequence[str] = BASE_FEATURES,
                                  max_gs_num: int = 100_000, remove_outlier_ndevs: float = 0.0
                                  ) -> Tuple[Dict[str, Tensor], MinMaxScaler]:
    """dataset/GS.py:153-204 -> (normalised Gaussian parameters, the fitted scaler)."""
    ckpt = torch.load(_last_checkpoint(nerfstudio_dir), map_location="cpu", weights_only=True)
    if "pipeline" in ckpt and isinstance(ckpt["pipeline"], dict):
        ckpt = ckpt["pipeline"]
    ckpt = {k.replace(GAUSS_PREFIX, ""): v for k, v in ckpt.items() if "gauss_params" in k}
    gs = {k: ckpt[k] for k in set(input_features)}
    # NaN rows (GS.py:166-174)
    select = torch.ones(gs["means"].shape[0], dtype=torch.bool)
    for k in gs:
        if k == "features_rest":
            select = select & ~torch.isnan(gs[k].sum(dim=1)).any(dim=1)
        else:
            select = select & ~torch.isnan(gs[k]).any(dim=1)
    gs = {k: v[select] for k, v in gs.items()}
    if remove_outlier_ndevs > 0:  # GS.py:177-180
        _, inl = remove_outliers(gs["means"], n_devs=remove_outlier_ndevs)
        gs = {k: v[inl] for k, v in gs.items()}
    n = gs["means"].shape[0]
    if n > max_gs_num:  # GS.py:183-188: keep the first max_gs_num
        gs = {k: v[:max_gs_num] for k, v in gs.items()}
    scaler = MinMaxScaler()
    gs["means"] = scaler.fit_transform(gs["means"])
    gs["scales"] = gs["scales"] + torch.log(scaler.scale_)
    inf_mask = torch.isinf(gs["scales"]).sum(dim=1).bool()
    inrange = torch.all((gs["means"] >= 0) & (gs["means"] <= 1), dim=1)
    valid = (~inf_mask) & inrange
    gs = {k: v[valid] for k, v in gs.items()}
    return gs, scaler


# ---- camera pickle -----------------------------------------------------------------------------------------
def _tensor_from_bytes(b: bytes):
    return torch.load(io.BytesIO(b), map_location="cpu", weights_only=True)


class _RestrictedUnpickler(pickle.Unpickler):
    """Builds containers, numbers, strings, numpy arrays and torch tensors; refuses every other global."""

    _NUMPY = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
              ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
              ("numpy._core.multiarray", "scalar")}
    _BUILTINS = {"dict", "list", "tuple", "set", "frozenset", "int", "float", "complex", "str", "bytes", "bool",
                 "slice", "range"}

    def find_class(self, module, name):
        if module == "builtins" and name in self._BUILTINS:
            return getattr(__import__("builtins"), name)
        if (module, name) in self._NUMPY:
            mod = __import__(module, fromlist=[name])
            return getattr(mod, name)
        if module == "collections" and name == "OrderedDict":
            import collections
            return collections.OrderedDict
        if module == "torch.storage" and name == "_load_from_bytes":
            return _tensor_from_bytes
        if module == "torch._utils" and name in ("_rebuild_tensor_v2", "_rebuild_tensor"):
            import torch._utils as tu
            return getattr(tu, name)
        raise pickle.UnpicklingError(f"camera pickle: refusing global {module}.{name}")


def load_camera_pickle(path: str) -> dict:
    with open(path, "rb") as f:
        return _RestrictedUnpickler(f).load()


def _as_tensor(x):
    return x if isinstance(x, Tensor) else torch.as_tensor(np.asarray(x))


def load_images_cameras_fromnerfstudio(nerfstudio_dir: str, colmap_dir: str) -> Tuple[dict, List[str], List[str]]:
    """dataset/GS.py:206-244: camera meta + train / test image paths with the OOD test-split rules."""
    meta = load_camera_pickle(os.path.join(nerfstudio_dir, "camera_for-3d-denoise.pkl"))
    names = os.listdir(os.path.join(colmap_dir, "images"))
    split_file = os.path.join(colmap_dir, "ood-test_split.txt")
    ood_names = None
    if os.path.isfile(split_file):
        with open(split_file) as f:
            ood_names = [ln.strip() for ln in f.readlines()]
    train, test = [], []
    elevation = False
    for name in sorted(names):
        if "elevation" in name:  # the synthetic OOD test set: elevation 70/80/90 only
            elevation = True
            if "elevation90" in name or "elevation80" in name or "elevation70" in name:
                test.append(os.path.join(colmap_dir, "images", name))
        elif name.startswith("test") or name.startswith("frame_eval"):
            test.append(os.path.join(colmap_dir, "images", name))
        else:
            train.append(os.path.join(colmap_dir, "images", name))
    if elevation:
        meta["test_camera_to_worlds"] = meta["test_camera_to_worlds"][-3 * 3:]
    if ood_names is not None:
        ids = [i for i, pth in enumerate(test) if os.path.basename(pth) in ood_names]
        test = [test[i] for i in ids]
        meta["test_camera_to_worlds"] = meta["test_camera_to_worlds"][ids]
    return meta, train, test


def load_scene(nerfstudio_dir: str, colmap_dir: str, input_features: Sequence[str] = BASE_FEATURES,
               max_gs_num: int = 100_000, remove_outlier_ndevs: float = 0.0,
               background_color: Sequence[float] = (0, 0, 0)) -> dict:
    """dataset/GS.py:308-322 + the camera dict of __iter__ (:392-395): normalised Gaussians and the test
    cameras (translations mapped by the Gaussians' scaler) in the renderer's `cameras` layout."""
    gs, scaler = load_gs_params_fromnerfstudio(nerfstudio_dir, input_features, max_gs_num, remove_outlier_ndevs)
    meta, train, test = load_images_cameras_fromnerfstudio(nerfstudio_dir, colmap_dir)
    for key in ("train_camera_to_worlds", "test_camera_to_worlds"):
        if key in meta:
            c2w = _as_tensor(meta[key]).clone()
            c2w[:, :3, -1] = scaler.transform(c2w[:, :3, -1])
            meta[key] = c2w
    cameras = {"camera_to_worlds": meta["test_camera_to_worlds"]}
    for key in ("fx", "fy", "cx", "cy", "width", "height"):
        cameras[key] = meta[key]
    cameras["background_color"] = torch.tensor(list(background_color), dtype=torch.float32) / 255.0
    return {"gs_params": gs, "meta": meta, "cameras": cameras, "scaler": scaler, "train_imgs_path": train,
            "test_imgs_path": test, "scene_name": os.path.normpath(nerfstudio_dir).split(os.sep)[-2]}


def read_image(path: str, background: Tensor) -> Tensor:
    """dataset/GS.py:128-151: float image in [0,1] (uint8 / 255); RGBA composited over `background`; for a
    'real' scene with a mask image (images -> masks), the RGB composited through the mask plus the mask as a
    fourth channel (kept for masked evaluation)."""
    from PIL import Image
    image = torch.from_numpy(np.array(Image.open(path), dtype="uint8").astype(np.float32) / 255.0)
    mask = None
    if "real" in path.lower():
        mpath = path.replace("images", "masks")
        if os.path.exists(mpath):
            mask = torch.from_numpy(np.array(Image.open(mpath)).astype(np.float32) / 255.0)
    if image.shape[2] == 4:
        image = image[:, :, :3] * image[:, :, -1:] + background * (1.0 - image[:, :, -1:])
    elif mask is not None:
        rgb = image * mask[..., None] + background * (1.0 - mask[..., None])
        image = torch.concat([rgb, mask[..., None]], axis=-1)
    return image
