"""Pointcept serialization restated in numpy (bit-exact integer arithmetic).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Pointcept (hchautran fork, un-vendored submodule: reference .gitmodules:1-3)
`pointcept/models/utils/serialization/{default.py,z_order.py,hilbert.py}` and
`Point.serialization` (structure.py), called at reference
models/pointtransformer_v3.py:380 with order=("z","z-trans","hilbert",
"hilbert-trans") (:130) and shuffle_orders=True (:146).  The Hilbert encoder
below is the literal bit-array formulation (Skilling 2004) Pointcept uses,
deliberately different in form from the integer-register kernel in
csrc/serialize.hip so the two check each other.
"""
from __future__ import annotations

import numpy as np

ORDER_TYPES = {"z": 0, "z-trans": 1, "hilbert": 2, "hilbert-trans": 3}


def _xyz2key_lut_part(x, y, z, depth):
    key = np.zeros_like(x)
    for i in range(depth):
        mask = 1 << i
        key = key | ((x & mask) << (2 * i + 2)) | ((y & mask) << (2 * i + 1)) | ((z & mask) << (2 * i + 0))
    return key


_R256 = np.arange(256, dtype=np.int64)
_ZERO = np.zeros(256, dtype=np.int64)
_EX = _xyz2key_lut_part(_R256, _ZERO, _ZERO, 8)
_EY = _xyz2key_lut_part(_ZERO, _R256, _ZERO, 8)
_EZ = _xyz2key_lut_part(_ZERO, _ZERO, _R256, 8)


def z_order_encode(grid: np.ndarray, depth: int) -> np.ndarray:
    """z_order.xyz2key (OCNN KeyLUT): 8-bit LUT chunks, upper chunk << 24."""
    x, y, z = grid[:, 0].astype(np.int64), grid[:, 1].astype(np.int64), grid[:, 2].astype(np.int64)
    mask = 255 if depth > 8 else (1 << depth) - 1
    key = _EX[x & mask] | _EY[y & mask] | _EZ[z & mask]
    if depth > 8:
        mask = (1 << (depth - 8)) - 1
        key16 = _EX[(x >> 8) & mask] | _EY[(y >> 8) & mask] | _EZ[(z >> 8) & mask]
        key = key16 << 24 | key
    return key


def _right_shift(binary, k):
    if binary.shape[-1] <= k:
        return np.zeros_like(binary)
    out = np.zeros_like(binary)
    out[..., k:] = binary[..., :-k]
    return out


def _gray2binary(gray):
    shift = 2 ** (int(np.ceil(np.log2(gray.shape[-1]))) - 1)
    while shift > 0:
        gray = np.logical_xor(gray, _right_shift(gray, shift))
        shift //= 2
    return gray


def hilbert_encode(grid: np.ndarray, depth: int) -> np.ndarray:
    """hilbert.encode(locs, num_dims=3, num_bits=depth): bit arrays MSB-first, Skilling transform."""
    num_dims, num_bits = 3, depth
    locs = grid.astype(np.int64)
    # bits of each coordinate, MSB-first, truncated to num_bits
    shifts = np.arange(num_bits - 1, -1, -1)
    gray = ((locs[:, :, None] >> shifts[None, None, :]) & 1).astype(bool)  # [N, dims, bits]
    for bit in range(num_bits):
        for dim in range(num_dims):
            mask = gray[:, dim, bit].copy()
            gray[:, 0, bit + 1:] = np.logical_xor(gray[:, 0, bit + 1:], mask[:, None])
            to_flip = np.logical_and(~mask[:, None], np.logical_xor(gray[:, 0, bit + 1:], gray[:, dim, bit + 1:]))
            gray[:, dim, bit + 1:] = np.logical_xor(gray[:, dim, bit + 1:], to_flip)
            gray[:, 0, bit + 1:] = np.logical_xor(gray[:, 0, bit + 1:], to_flip)
    gray = gray.swapaxes(1, 2).reshape(-1, num_bits * num_dims)
    hh = _gray2binary(gray)
    L = hh.shape[1]
    weights = (np.int64(1) << np.arange(L - 1, -1, -1, dtype=np.int64))
    return (hh.astype(np.int64) * weights[None]).sum(1)


def encode(grid: np.ndarray, batch: np.ndarray | None, depth: int, order: str) -> np.ndarray:
    """serialization.encode: per-order code | batch << 3*depth."""
    if order == "z":
        code = z_order_encode(grid, depth)
    elif order == "z-trans":
        code = z_order_encode(grid[:, [1, 0, 2]], depth)
    elif order == "hilbert":
        code = hilbert_encode(grid, depth)
    elif order == "hilbert-trans":
        code = hilbert_encode(grid[:, [1, 0, 2]], depth)
    else:
        raise NotImplementedError(order)
    if batch is not None:
        code = (batch.astype(np.int64) << (depth * 3)) | code
    return code


def serialization(grid: np.ndarray, batch: np.ndarray, orders=("z", "z-trans", "hilbert", "hilbert-trans"),
                  perm=None, depth=None):
    """Point.serialization: codes [k,N], order = stable argsort, inverse; rows permuted by `perm`."""
    if depth is None:
        depth = int(grid.max()).bit_length()
    assert depth * 3 + len(np.unique(batch)).bit_length() <= 63 and depth <= 16
    code = np.stack([encode(grid, batch, depth, o) for o in orders])
    order = np.argsort(code, axis=1, kind="stable")
    inverse = np.zeros_like(order)
    rows = np.arange(code.shape[0])[:, None]
    inverse[rows, order] = np.arange(code.shape[1])[None]
    if perm is not None:
        perm = np.asarray(perm)
        code, order, inverse = code[perm], order[perm], inverse[perm]
    return code, order, inverse, depth
