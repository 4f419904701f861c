"""Build the libsfx C-ABI shared library (HIP, gfx950) in-tree.

`python -m splatformer_amd.build_lib` compiles every `csrc/*.hip` with hipcc for
gfx950 and links `splatformer_amd/libsfx.so`.  Objects are cached under
`build/` and only rebuilt when their source or a header changed.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
ROOT = os.path.dirname(HERE)
BUILD = os.path.join(ROOT, "build", "sfx")
LIB = os.path.join(HERE, "libsfx.so")
ARCH = os.environ.get("SFX_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

CFLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-fPIC",
    "-std=c++17",
    "-ffp-contract=fast-honor-pragmas",  # fused multiply-add except in `#pragma clang fp contract(off)` bodies
    "-munsafe-fp-atomics",
    "-Wno-unused-result",
    f"-I{CSRC}",
    f"-I{os.path.join(ROOT, 'include')}",
]


_INC = re.compile(r'^\s*#\s*include\s*"([^"]+)"', re.M)


def _deps_mtime(path: str, seen=None) -> float:
    """Newest mtime of `path` and of the in-tree headers it includes (transitively): an object is rebuilt only when
    one of ITS sources changed, not on every header edit (the gfx950 compile of the larger kernels takes minutes)."""
    seen = set() if seen is None else seen
    if path in seen or not os.path.exists(path):
        return 0.0
    seen.add(path)
    t = os.path.getmtime(path)
    for inc in _INC.findall(open(path, errors="ignore").read()):
        for d in (os.path.dirname(path), CSRC, os.path.join(ROOT, "include")):
            cand = os.path.join(d, inc)
            if os.path.exists(cand):
                t = max(t, _deps_mtime(cand, seen))
                break
    return t


def _flags_stamp() -> float:
    """mtime of a stamp file rewritten whenever the compile flags change (so a flag change rebuilds)."""
    stamp = os.path.join(BUILD, "flags.txt")
    want = " ".join([HIPCC, *CFLAGS])
    have = open(stamp).read() if os.path.exists(stamp) else None
    if have != want:
        with open(stamp, "w") as f:
            f.write(want)
    return os.path.getmtime(stamp)


def _compile(src: str, flags_mtime: float) -> str:
    obj = os.path.join(BUILD, os.path.basename(src).replace(".hip", ".o"))
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(_deps_mtime(src), flags_mtime):
        return obj
    cmd = [HIPCC, *CFLAGS, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build(verbose: bool = False, jobs: int | None = None) -> str:
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    hm = _flags_stamp()
    jobs = jobs or min(8, len(srcs))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hm), srcs))
    newest = max(os.path.getmtime(o) for o in objs)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < newest:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
