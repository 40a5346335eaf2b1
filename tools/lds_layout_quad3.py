"""Vectorised search for the 4-wave kernel's exchange map (see lds_layout_quad.py): weights
w_i = 2^i + d_i, d_i in [0, 16), scored per b128 instruction with the gfx950 lane groups."""
import itertools
import sys

import numpy as np

RG = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
      list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
RG += [[l + 32 for l in g] for g in RG]
WG = [list(range(i, i + 8)) for i in range(0, 64, 8)]


def mk(lane_bits, reg_bits):
    idx = np.zeros((2, 8, 64), np.int64)
    for h in range(2):
        for r in range(8):
            for L in range(64):
                v = 512 * h
                for k, b in enumerate(lane_bits):
                    v |= ((L >> k) & 1) << b
                for k, b in enumerate(reg_bits):
                    v |= ((r >> k) & 1) << b
                idx[h, r, L] = v
    return idx


def bits(idx):
    return np.stack([(idx >> i) & 1 for i in range(10)], -1)  # [..., 10]


def cost(addr, write):
    groups, ns = (WG, 8) if write else (RG, 16)
    tot = 0.0
    for g in groups:
        a = addr[..., g]  # [2, 8, glen]
        s = a % ns
        # conflict degree = max over slots of distinct addresses in that slot
        m = np.zeros(a.shape[:-1], np.int64)
        for sl in range(ns):
            mask = s == sl
            cnt = mask.sum(-1)  # addresses are distinct within an instruction here
            m = np.maximum(m, cnt)
        tot += m.sum()
    return tot / 16 / (8 if write else 4)


A = mk([0, 1, 2, 3, 4, 5], [7, 8, 9])
A[:, :, :] = np.array([[[128 * r + 64 * h + L for L in range(64)] for r in range(8)] for h in range(2)])


def run(Bl, Cl):
    Bm, Cm = mk(Bl, [4, 5, 6]), mk(Cl, [1, 2, 3])
    bA, bB, bC = bits(A), bits(Bm), bits(Cm)
    rng = np.random.default_rng(5)
    best = []
    allidx = bits(np.arange(1024))
    for trial in range(40000):
        d = rng.integers(0, 16, 10) * (rng.random(10) < 0.6)
        w = (1 << np.arange(10)) + d
        ad = allidx @ w
        if ad.max() >= 1088 or len(np.unique(ad)) != 1024:
            continue
        fA, fB, fC = bA @ w, bB @ w, bC @ w
        sc = (cost(fA, 1) + cost(fA, 0)) + 2 * (cost(fB, 1) + cost(fB, 0)) + (cost(fC, 1) + cost(fC, 0))
        best.append((sc, int(ad.max()), w.tolist()))
    best.sort()
    w = np.array(best[0][2])
    parts = {k: (cost(bits(m) @ w, 1), cost(bits(m) @ w, 0)) for k, m in (("A", A), ("B", Bm), ("C", Cm))}
    return best[0], parts


if __name__ == "__main__":
    for Bl, Cl in [((0, 1, 2, 3, 7, 8), (0, 4, 5, 6, 7, 8)), ((0, 1, 2, 3, 7, 8), (4, 5, 6, 7, 0, 8)),
                   ((0, 1, 2, 3, 7, 8), (4, 5, 6, 7, 8, 0)), ((7, 8, 0, 1, 2, 3), (4, 5, 6, 7, 0, 8))]:
        b, parts = run(Bl, Cl)
        print(Bl, Cl, b, {k: tuple(round(x, 2) for x in v) for k, v in parts.items()}, flush=True)
