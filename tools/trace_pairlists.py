"""Print where each PairLists of one config-B refine is created and where every HostRead value is first read, and
whether that read waited (GPU only): python tools/trace_pairlists.py"""
import os
import sys
import traceback

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from splatformer_amd import _lib, ptv3_ops as ops  # noqa: E402
from splatformer_amd.feature_predictor import FeaturePredictor  # noqa: E402
from splatformer_amd.scenes import make_scene, to_device  # noqa: E402

LOG = []


def where(skip=2):
    fr = [f for f in traceback.extract_stack()[:-skip] if "splatformer_amd" in f.filename]
    return " < ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in reversed(fr[-4:]))


_pl_init = ops.PairLists.__init__


def pl_init(self, nbr, centre):
    LOG.append(f"PairLists(n={nbr.shape[0]}, centre={centre}) at {where()}")
    _pl_init(self, nbr, centre)


_get = _lib.HostRead.get


def get(self):
    if self._v is None:
        LOG.append(f"  HostRead.get ({'ready' if self._ev.query() else 'WAITS'}) at {where()}")
    return _get(self)


ops.PairLists.__init__ = pl_init
_lib.HostRead.get = get

dev = torch.device("cuda")
torch.manual_seed(0)
model = FeaturePredictor(sh_degree=1, zeroinit=False).eval().to(dev)
scene = to_device(make_scene(100_000, sh_degree=1, seed=0), dev)
model.refine_packed(scene)
torch.cuda.synchronize()
LOG.clear()
model.refine_packed(scene)
torch.cuda.synchronize()
print("# model.refine_packed(scene)")
print("\n".join(LOG))
LOG.clear()
model([scene], [0])
torch.cuda.synchronize()
print("# model([scene], [0]) (bench.py's step)")
print("\n".join(LOG))
