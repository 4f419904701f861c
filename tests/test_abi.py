"""The C-ABI library loads (no GPU needed) and exports every symbol include/sfx.h declares."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "sfx.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sfx_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "sfx_rasterize_fwd" in syms and "sfx_sort_pairs_u64" in syms
    assert len(syms) >= 15


def test_library_exports_all_declared_symbols():
    from splatformer_amd import _lib
    lib = _lib.load()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, f"libsfx.so lacks: {missing}"
    assert lib.sfx_abi_version() == 16


def test_python_signatures_cover_header():
    from splatformer_amd import _lib
    import splatformer_amd.ptv3_ops  # noqa: F401  (registers the PTv3 entry points)
    import splatformer_amd.train_ops  # noqa: F401  (training entry points)
    import splatformer_amd.metrics  # noqa: F401  (evaluation entry points)
    import splatformer_amd.gs_render  # noqa: F401  (batched-view render entry points)
    import splatformer_amd.downsample  # noqa: F401  (point-downsampling entry points)
    missing = [s for s in declared_symbols() if s not in _lib.SIGNATURES]
    assert not missing, f"no ctypes signature for: {missing}"


def test_invalid_args_report_errors_without_gpu():
    """Argument validation runs host-side and fails with a message (no kernel launched)."""
    from splatformer_amd import _lib
    lib = _lib.load()
    rc = lib.sfx_project_fwd(-1, None, None, 1.0, None, None, 1.0, 1.0, 0.0, 0.0, 8, 8, 16, 0.01,
                             None, None, None, None, None, None, None, None)
    assert rc == -1
    assert b"n < 0" in lib.sfx_last_error()
    rc = lib.sfx_sort_pairs_u64(10, None, None, None, None, 0, 70, None, 0, None)
    assert rc == -1
    assert b"bit range" in lib.sfx_last_error()


def test_no_cpu_fallback_on_cpu_tensors():
    import torch
    from splatformer_amd import gsplat_compat
    with pytest.raises(RuntimeError):
        gsplat_compat.spherical_harmonics(1, torch.randn(4, 3), torch.randn(4, 4, 3))
