"""CPU oracle for the SplatFormer refine+render hot path.

TEST INFRASTRUCTURE ONLY.  Only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` may import this package, and only as the
checker / the timed CPU baseline -- never as the product path.  The product
(`splatformer_amd`) never imports it and has no CPU fallback.

Contents (each function cites the reference file:line it restates):
  * gsplat_ref   -- gsplat v0.1.11 SH / projection / binning / rasterize
                    forward+backward (un-vendored dependency, README.md:27;
                    called at utils/gs_utils.py:78, :82-95, :96-109).
  * serialize_ref -- Pointcept z-order / Hilbert serialization (numpy,
                    bit-exact integer arithmetic).
  * ptv3_ref     -- Pointcept PTv3 m1 modules (Block, SerializedAttention,
                    SubMConv3d, pooling/unpooling) as used by
                    models/pointtransformer_v3.py, plus the FeaturePredictor
                    heads of models/feature_predictor.py.
  * render_ref   -- utils/gs_utils.py:29-114 render glue.

Parity status: the glue (gs_utils.py, feature_predictor.py) is pinned by
golden vectors captured from the reference itself (tests/golden/).  The
gsplat / Pointcept / spconv arithmetic lives in third-party code absent from
/root/reference; it is restated from the published v0.1.11 / PTv3-m1 sources
and pinned by known-answer tests only ("parity unpinned" against the real
dependency).
"""
