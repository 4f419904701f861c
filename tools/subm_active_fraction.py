"""MFMA padding of an output-row-stationary SubM conv on the config-B stage geometries (CPU, numpy): for each stage
map, the rows a conv that skips (group, offset) pairs with no neighbour computes, over the pair products it needs
(n + pairs), at 16- and 32-row groups, for rows in input order, in serialized (z-order) order, and sorted by their
neighbour mask (the rarest offsets -- corners, then edges, then faces -- in the key's high bits, all 26 bits or
the 16 bits sfx_subm_order_keys uses).  usage: python tools/subm_active_fraction.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splatformer_amd.scenes import make_scene  # noqa: E402

OFFS = np.array([(i, j, k) for i in (-1, 0, 1) for j in (-1, 0, 1) for k in (-1, 0, 1)])
CLS = np.abs(OFFS).sum(1)
KEY26 = [k for c in (3, 2, 1) for k in range(27) if CLS[k] == c]   # MSB first
KEY16 = [2, 6, 8, 18, 20, 24, 26, 1, 7, 9, 11, 15, 17, 23, 10, 12]  # subm_fused.hip kOrderBits


def active(g):
    key = lambda a: (a[:, 0] + 2) * (1 << 40) + (a[:, 1] + 2) * (1 << 20) + (a[:, 2] + 2)
    uk = np.unique(key(g))
    act = np.zeros((len(g), 27), bool)
    for o in range(27):
        kk = key(g + OFFS[o])
        pos = np.clip(np.searchsorted(uk, kk), 0, len(uk) - 1)
        act[:, o] = uk[pos] == kk
    return act


def zorder(g):
    k = np.zeros(len(g), np.int64)
    for b in range(21):
        for a in range(3):
            k |= ((g[:, a] >> b) & 1) << (3 * b + a)
    return k


def padding(act, rows, B):
    a = act[rows]
    n = len(a)
    nb = (n + B - 1) // B
    a = np.concatenate([a, np.zeros((nb * B - n, 27), bool)]).reshape(nb, B, 27)
    return a.any(1).sum() * B / act.sum()


def main():
    grid = np.floor(make_scene(100000, 1, seed=0)["means"].numpy() * 384).astype(np.int64)
    g = grid
    print("stage      n  pairs/pt | B   input  z-order  mask26  mask16")
    for s, pd in enumerate([None, 0, 1, 1, 1]):
        if pd is not None:
            g = np.unique(g >> pd, axis=0)
        act = active(g)
        n = len(g)
        orders = {"input": np.arange(n), "z": np.argsort(zorder(g), kind="stable")}
        for name, bits in (("m26", KEY26), ("m16", KEY16)):
            key = np.zeros(n, np.int64)
            for b in bits:
                key = (key << 1) | act[:, b]
            orders[name] = np.argsort(key, kind="stable")
        for B in (16, 32):
            vals = [padding(act, orders[k], B) for k in ("input", "z", "m26", "m16")]
            print(f"s{s} {n:7d} {(act.sum() - n) / n:8.2f} | {B:2d} " + " ".join(f"{v:7.3f}" for v in vals))


if __name__ == "__main__":
    main()
