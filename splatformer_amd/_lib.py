"""ctypes binding of the libsfx C-ABI (include/sfx.h).

The product path has exactly one implementation: the HIP kernels in
`libsfx.so`.  If the library is missing, or no GPU is visible, every op raises
immediately -- there is no CPU fallback.  (The CPU restatement under
`oracle/` is test infrastructure only and is never imported from here.)
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SFX_LIB", os.path.join(_HERE, "libsfx.so"))

P = C.c_void_p
I = C.c_int
L = C.c_longlong
F = C.c_float
Z = C.c_size_t

# name -> argtypes (restype int unless listed in _RESTYPES)
SIGNATURES: dict[str, list] = {
    "sfx_abi_version": [],
    "sfx_last_error": [],
    "sfx_scan_workspace_bytes": [L],
    "sfx_lookback_timeouts": [P],
    "sfx_lookback_release": [P],
    "sfx_scan_i32": [L, P, P, I, P, Z, P, P],
    "sfx_scan_i64": [L, P, P, I, P, Z, P, P],
    "sfx_sort_workspace_bytes": [L],
    "sfx_sort_pairs_u64": [L, P, P, P, P, I, I, P, Z, P],
    "sfx_sh_fwd": [I, I, I, P, P, P, P],
    "sfx_sh_bwd": [I, I, I, P, P, P, P],
    "sfx_project_fwd": [I, P, P, F, P, P, F, F, F, F, I, I, I, F, P, P, P, P, P, P, P, P],
    "sfx_project_bwd": [I, P, P, F, P, P, F, F, P, P, P, P, P, P, P, P, P, P, P, P, P, P],
    "sfx_render_prep_project": [I, I, P, L, P, L, P, L, P, L, P, L, P, L, P, F, F, F, F, I, I, I, P, P, P, P, P, P, P,
                                P, P],
    "sfx_isect_emit": [I, P, P, P, P, I, I, I, P, P, P],
    "sfx_tile_bins": [I, P, I, P, P],
    "sfx_profile_marker": [I, P],
    "sfx_rasterize_fwd": [I, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P],
    "sfx_rasterize_bwd": [I, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P],
}
_RESTYPES = {
    "sfx_abi_version": C.c_int,
    "sfx_last_error": C.c_char_p,
    "sfx_scan_workspace_bytes": C.c_size_t,
    "sfx_lookback_timeouts": C.c_longlong,
    "sfx_sort_workspace_bytes": C.c_size_t,
}

_lib = None
_lock = threading.Lock()


def register(name: str, argtypes: list, restype=C.c_int) -> None:
    """Extend the signature table (used by modules that add entry points)."""
    SIGNATURES[name] = argtypes
    if restype is not C.c_int:
        _RESTYPES[name] = restype


def load(path: str | None = None):
    """Load libsfx.so (no GPU needed); raises if it is absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise RuntimeError(
                f"libsfx.so not found at {p}; build it with `python -m splatformer_amd.build_lib` "
                "(the HIP extension is required: there is no CPU fallback)")
        lib = C.CDLL(p)
        for name, args in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = _RESTYPES.get(name, C.c_int)
        _lib = lib
        return lib


def lib():
    return _lib if _lib is not None else load()


def fn(name: str):
    l = lib()
    f = getattr(l, name)
    if f.argtypes is None and name in SIGNATURES:
        f.argtypes = SIGNATURES[name]
        f.restype = _RESTYPES.get(name, C.c_int)
    return f


_FNS: dict = {}  # name -> resolved ctypes function (one dict lookup per launch instead of lib() + getattr + checks)


def call(name: str, *args) -> None:
    f = _FNS.get(name)
    if f is None:
        f = _FNS[name] = fn(name)
    rc = f(*args)
    if rc != 0:
        msg = lib().sfx_last_error()
        raise RuntimeError(f"{name} failed ({rc}): {msg.decode() if msg else ''}")


class HostRead:
    """Asynchronous device -> pinned-host copy of a small tensor: `get()` waits only for the work enqueued before
    the copy, so GPU work enqueued between the two keeps the device busy while the host waits (the sizes that
    must reach the host -- pooled point counts, pair offsets, the grid depth -- cost no queue drain)."""

    def __init__(self, t: torch.Tensor):
        self._h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        self._h.copy_(t, non_blocking=True)
        self._ev = torch.cuda.Event()
        self._ev.record()
        self._v = None

    def get(self) -> list:
        if self._v is None:
            self._ev.synchronize()
            self._v = self._h.tolist()
        return self._v

    def ready(self) -> bool:
        """Whether get() would return without waiting."""
        return self._v is not None or self._ev.query()


_LB_SEEN: dict = {}  # stream -> look-back timeouts already reported (one process per GPU)


def check_lookback(where: str, st=None) -> None:
    """Raise if a decoupled look-back wait (single-pass scan / radix pass, csrc/common.h lb_lookback_wave) on this
    stream reached its spin cap since the last check: that scan's prefix -- an intersection list, a pooled count --
    is wrong.  Call where results are consumed on the host (the stream is drained there anyway: the call
    synchronises it).  Each timeout is reported once; later checks only report new ones."""
    st = stream() if st is None else st
    n = int(fn("sfx_lookback_timeouts")(st))
    if n <= 0:  # 0: every wait exact; -1: nothing scanned on this stream yet
        return
    seen = _LB_SEEN.get(st, 0)
    if n > seen:
        _LB_SEEN[st] = n
        raise RuntimeError(f"{where}: {n - seen} decoupled look-back wait(s) on this stream reached the spin cap "
                           "(a scan or radix pass produced a wrong prefix; its results are invalid)")


def require_gpu(t: torch.Tensor | None = None) -> None:
    if not torch.cuda.is_available():
        raise RuntimeError("splatformer_amd requires a ROCm GPU (MI355X); no device is visible")
    if t is not None and not t.is_cuda:
        raise RuntimeError("splatformer_amd ops take device tensors; got a CPU tensor")


def ptr(t: torch.Tensor | None, dtype: torch.dtype | None = None) -> int | None:
    """Device pointer of a contiguous tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("expected a device tensor")
    if not t.is_contiguous():
        raise RuntimeError("expected a contiguous tensor")
    if dtype is not None and t.dtype != dtype:
        raise RuntimeError(f"expected dtype {dtype}, got {t.dtype}")
    return t.data_ptr()


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_get_device = torch._C._cuda_getDevice
_cuda_ready = [False]


def stream() -> int:
    """The current HIP stream of the current device (torch's), as a pointer.  Called once per launch: the raw
    accessor costs ~0.3 us against ~8 us for torch.cuda.current_stream()'s Python wrapper (tools/host_profile.py)."""
    if _raw_stream is not None:
        if _cuda_ready[0] or torch.cuda.is_initialized():
            _cuda_ready[0] = True
            return _raw_stream(_get_device())
    return torch.cuda.current_stream().cuda_stream


def workspace(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)
