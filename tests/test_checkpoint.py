"""Checkpoint compatibility: a reference-style FeaturePredictor checkpoint (DDP
`module.` prefix, SyncBN keys, spconv 1.x conv layout) loads into this build's module with every key matched
and the derived (folded / packed) weights rebuilt.  CPU only (no kernel calls)."""
import os

import torch

from splatformer_amd.feature_predictor import FeaturePredictor, convert_state_dict, load_checkpoint


def test_reference_checkpoint_roundtrip(tmp_path):
    torch.manual_seed(0)
    src = FeaturePredictor(sh_degree=1, zeroinit=False)
    sd = src.state_dict()
    # what train.py:344 writes for a DDP(SyncBN(model)) run, with an spconv 1.x conv layout on top
    ref = {}
    for k, v in sd.items():
        v = v.clone()
        if v.dim() == 5:
            v = v.permute(1, 2, 3, 4, 0).contiguous()  # [Cout,3,3,3,Cin] -> [3,3,3,Cin,Cout]
        ref["module." + k] = v
    path = os.path.join(str(tmp_path), "train-on-objaverse.pth")
    torch.save(ref, path)
    torch.manual_seed(1)
    dst = FeaturePredictor(sh_degree=1, zeroinit=True, resume_ckpt=path)
    for k, v in dst.state_dict().items():
        assert torch.equal(v, sd[k]), k
    # the reference's own key set: backbone.* + features_outputhead.<feature>.<layer>.* (feature_predictor.py)
    keys = set(dst.state_dict())
    assert any(k.startswith("backbone.backbone.enc.enc0.block0.cpe.0.weight") for k in keys)
    assert "features_outputhead.means.0.weight" in keys and "features_outputhead.quats.6.bias" in keys
    conv = [k for k in keys if k.endswith("cpe.0.weight")]
    assert len(conv) == 22 and all(dst.state_dict()[k].shape[1:4] == (3, 3, 3) for k in conv)


def test_load_checkpoint_strict_reports_missing():
    m = FeaturePredictor(sh_degree=1)
    sd = m.state_dict()
    sd.pop("features_outputhead.means.0.weight")
    try:
        load_checkpoint(m, sd)
    except RuntimeError as e:
        assert "features_outputhead.means.0.weight" in str(e)
    else:
        raise AssertionError("strict load accepted a missing key")
    assert convert_state_dict({}, {}) == {}


def test_pretrained_backbone_checkpoint(tmp_path):
    """pointtransformer_v3.py:164-178: a Pointcept segmentor checkpoint ({'state_dict': {'module.backbone.*',
    'module.seg_head.*'}}, e.g. a ScanNet PTv3 with 6 input channels) feeds the backbone -- keys matched by name
    after stripping 'module.backbone.', shape mismatches (the embedding) and non-backbone keys skipped, nothing
    else touched.  The checkpoint is built from a module of a different configuration (in_channels 6), not from
    the module that loads it."""
    from splatformer_amd.ptv3 import PointTransformerV3Model
    torch.manual_seed(3)
    scannet = PointTransformerV3Model(in_channels=6)
    sd = {"module.backbone." + k: v.clone() for k, v in scannet.backbone.state_dict().items()}
    sd["module.seg_head.weight"] = torch.randn(20, 64)
    sd["module.seg_head.bias"] = torch.randn(20)
    path = os.path.join(str(tmp_path), "scannet-semseg-pt-v3m1-0-base.pth")
    torch.save({"state_dict": sd, "epoch": 100}, path)
    torch.manual_seed(4)
    fresh = PointTransformerV3Model(in_channels=23)
    before = {k: v.clone() for k, v in fresh.backbone.state_dict().items()}
    torch.manual_seed(4)
    loaded = PointTransformerV3Model(in_channels=23, pretrained_ckpt=path)
    src = scannet.backbone.state_dict()
    n_loaded = n_skipped = 0
    for k, v in loaded.backbone.state_dict().items():
        if src[k].shape == v.shape:
            assert torch.equal(v, src[k]), k
            n_loaded += 1
        else:  # the embedding's input width differs (6 vs 23): left at its own initialisation
            assert torch.equal(v, before[k]), k
            n_skipped += 1
    assert n_skipped >= 1 and n_loaded > 100
    assert all(k.startswith("embedding") for k, v in loaded.backbone.state_dict().items() if src[k].shape != v.shape)
