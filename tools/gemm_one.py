"""One dense sfx_linear shape, launched `reps` times back to back (PMC passes / quick timing; GPU only):
python tools/gemm_one.py M N K reps [act]   (act: none | gelu)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splatformer_amd import ptv3_ops as ops  # noqa: E402

M, N, K, reps = (int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (37759, 1024, 256, 20)))
act = sys.argv[5] if len(sys.argv) > 5 else "none"
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(M, K, device=dev, generator=g)
w = torch.randn(N, K, device=dev, generator=g) * K ** -0.5
b = torch.randn(N, device=dev, generator=g)
kw = dict(act=ops.ACT_GELU) if act == "gelu" else {}
ops.linear(x, w, b, **kw)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    ops.linear(x, w, b, **kw)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / reps
print(f"M={M} N={N} K={K} {act}: {us:.1f} us/call {2.0 * M * N * K / us / 1e6:.1f} TF/s")
if os.environ.get("SFX_WS_TRACE_READ"):
    import ctypes as C
    from splatformer_amd import _lib
    lib = _lib.load()
    buf = (C.c_ulonglong * 16)()
    lib.sfx_ws_trace(buf, 0)
    names = ["p_issue", "p_store", "p_epi", "p_bar", "c_pre", "c_mma", "c_stage", "c_bar"]
    rounds = buf[8]
    print("per round (cycles, summed over WGs / rounds):",
          {n: round(buf[i] / max(1, rounds), 1) for i, n in enumerate(names)})
