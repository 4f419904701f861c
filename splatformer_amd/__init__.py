"""splatformer_amd: MI355X-native (gfx950) SplatFormer refine+render hot path.

Host side mirrors the reference interfaces (gsplat v0.1.11 API, Pointcept
PTv3 module API, FeaturePredictor); every op runs on the HIP kernels of the
in-tree C-ABI library `libsfx.so` (include/sfx.h).  No CPU fallback.
"""
__version__ = "0.1.0"
