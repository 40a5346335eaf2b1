#!/usr/bin/env python3
"""CPU emulation of br_qy.hip's data movement (no GPU): the forward transform phases A -> B -> B' -> E
and the inverse E -> B' -> B -> A, transcribed from the kernel (registers, v_permlane32/16_swap as lane
swaps, the LDS map xq, the zeta / twiddle table indexing), checked against the oracle's transforms
(oracle/tfhe_oracle.c forward_twisted, fho_fft_inverse) in numpy complex128.
usage: python3 tools/qy_emulate.py"""
import numpy as np

XW = [8, 2, 1, 4, 16, 32, 68, 135, 280, 550]
QP = [9, 5, 8, 7, 6, 1]
QE = [5, 4, 8, 7, 6, 9]
QW1, QW0 = 2, 3


def bt(v, k):
    return (v >> k) & 1


def xq(idx):
    return sum(XW[k] for k in range(10) if idx >> k & 1)


def idx_B(h, L, r):
    return (bt(r, 2) << 6) | (bt(r, 1) << 5) | (bt(r, 0) << 7) | (bt(L, 5) << 9) | (bt(L, 4) << 8) | ((L & 15) << 1) | h


def idx_Bp(h, L, r):
    v = (bt(r, 2) << 4) | (bt(r, 1) << 3) | (bt(r, 0) << 2) | h
    for m in range(6):
        v |= bt(L, 5 - m) << QP[m]
    return v


def idx_E(e, L, k):
    v = (bt(e, 1) << QW1) | (bt(e, 0) << QW0) | (bt(k, 1) << 1) | bt(k, 0)
    for m in range(6):
        v |= bt(L, 5 - m) << QE[m]
    return v


def bitrev(b, bits):
    return int(format(b, f"0{bits}b")[::-1], 2) if bits else 0


ZETA = np.zeros(1024, complex)
for st in range(10):
    for b in range(0, 1 << st, 2):
        ZETA[(1 << st) + b] = np.exp(1j * np.pi * (4 * bitrev(b, st) + 1) / (1 << (st + 2)))
        if st > 0:
            ZETA[(1 << st) + b + 1] = 1j * ZETA[(1 << st) + b]
W = np.exp(2j * np.pi * np.arange(512) / 1024)


def ref_forward(x):
    x = x.copy()
    for st in range(10):
        h = 512 >> st
        for b in range(1 << st):
            z = ZETA[(1 << st) + b]
            for j in range(h):
                p, q = 2 * h * b + j, 2 * h * b + j + h
                a, c = x[p], x[q]
                x[p], x[q] = a + z * c, a - z * c
    return x


def ref_inverse(x):
    x = x.copy()
    for s in range(9, -1, -1):
        h = 512 >> s
        for b in range(0, 1024, 2 * h):
            for j in range(h):
                w = np.conj(W[j << s])
                a, c = x[b + j], x[b + j + h]
                x[b + j], x[b + j + h] = a + w * c, a - w * c
    return x


def bfly(x, i, j, w):  # dit_bfly: (a, c) -> (a + w c, a - w c)
    a, c = x[i], x[j]
    x[i], x[j] = a + w * c, a - w * c


def permlane(X, Y, K):
    """register pair (X, Y) = register bit 0 / 1 <-> lane bit K (v_permlane32/16_swap)"""
    m = 1 << K
    for L in range(64):
        if L & m:
            X[L], Y[L ^ m] = Y[L ^ m], X[L]


def mul_i(z):
    return 1j * z


def main():
    rng = np.random.default_rng(5)
    poly = [rng.standard_normal(1024) + 1j * rng.standard_normal(1024) for _ in range(2)]
    # x[w][r] = array over 64 lanes
    x = [[np.array([poly[w >> 1][128 * r + 2 * L + (w & 1)] for L in range(64)]) for r in range(8)] for w in range(4)]
    s_z = np.zeros(140, complex)
    for k in range(140):
        if k < 4: zi = 8 + 2 * k
        elif k < 12: zi = 16 + 2 * (k - 4)
        elif k < 44: zi = 32 + (k - 12)
        elif k < 76: zi = 64 + 2 * (k - 44)
        else: zi = 128 + 4 * ((k - 76) & 31) + 2 * ((k - 76) >> 5)
        s_z[k] = ZETA[zi]
    XR = sum(XW) + 1
    lds = np.full(2 * XR, np.nan + 0j)
    Lv = np.arange(64)
    for w in range(4):
        p, h = w >> 1, w & 1
        X = x[w]
        for r in range(4): bfly(X, r, r + 4, ZETA[1])
        for r in range(8):
            if not r & 2: bfly(X, r, r + 2, mul_i(ZETA[2]) if r >> 2 else ZETA[2])
        for r in range(0, 8, 2):
            base = ZETA[6] if r >> 2 else ZETA[4]
            bfly(X, r, r + 1, mul_i(base) if (r >> 1) & 1 else base)
        for r in range(4): permlane(X[r], X[r + 4], 5)
        for r in range(8):
            if not r & 2: permlane(X[r], X[r + 2], 4)
        k98 = 2 * ((Lv >> 5) & 1) + ((Lv >> 4) & 1)
        z3, z4a, z4b = s_z[k98], s_z[4 + 2 * k98], s_z[5 + 2 * k98]
        for r in range(4): bfly(X, r, r + 4, mul_i(z3) if r & 1 else z3)
        for r in range(8):
            if r & 2: continue
            base = z4b if r & 1 else z4a
            bfly(X, r, r + 2, mul_i(base) if r >> 2 else base)
        for r in range(8):
            for L in range(64): lds[p * XR + xq(idx_B(h, L, r))] = X[r][L]
        for r in range(8):
            X[r] = np.array([lds[p * XR + xq(idx_Bp(h, L, r))] for L in range(64)])
        ip = np.array([idx_Bp(h, L, 0) for L in range(64)])
        U = ip >> 5
        z5, z6, z7a, z7b = s_z[12 + U], s_z[44 + U], s_z[76 + U], s_z[108 + U]
        for r in range(4): bfly(X, r, r + 4, z5)
        for r in range(8):
            if not r & 2: bfly(X, r, r + 2, mul_i(z6) if r & 4 else z6)
        for r in range(0, 8, 2):
            base = z7b if r & 4 else z7a
            bfly(X, r, r + 1, mul_i(base) if r & 2 else base)
        for r in range(8):
            for L in range(64): lds[p * XR + xq(idx_Bp(h, L, r))] = X[r][L]
    # phase E
    ref = [ref_forward(poly[p]) for p in range(2)]
    err = 0.0
    E = []
    for w in range(4):
        ie = np.array([idx_E(w, L, 0) for L in range(64)])
        V = ie >> 2
        z8, z9 = ZETA[256 + V], ZETA[512 + 2 * V]
        X = [np.array([lds[(r >> 2) * XR + xq(idx_E(w, L, r & 3))] for L in range(64)]) for r in range(8)]
        for r in range(8):
            if not r & 2: bfly(X, r, r + 2, z8)
        for r in range(0, 8, 2): bfly(X, r, r + 1, mul_i(z9) if r & 2 else z9)
        for r in range(8):
            got = X[r]
            want = np.array([ref[r >> 2][idx_E(w, L, r & 3)] for L in range(64)])
            err = max(err, np.abs(got - want).max())
        E.append(X)
    print(f"forward: max |kernel layout - oracle forward_twisted| = {err:.3e}")
    assert err < 1e-9
    # inverse: feed the forward outputs back (no MAC), expect fho_fft_inverse of them
    inv_ref = [ref_inverse(ref[p]) for p in range(2)]
    lds[:] = np.nan
    for w in range(4):
        X = E[w]
        for r in range(0, 8, 2):
            a0, c0 = X[r].copy(), X[r + 1].copy()
            X[r], X[r + 1] = a0 + c0, a0 - c0
        for r in range(8):
            if r & 2: continue
            t = -1j * X[r + 2] if r & 1 else X[r + 2]
            a = X[r].copy()
            X[r], X[r + 2] = a + t, a - t
        for r in range(8):
            for L in range(64): lds[(r >> 2) * XR + xq(idx_E(w, L, r & 3))] = X[r][L]
    err = 0.0
    for w in range(4):
        p, h = w >> 1, w & 1
        X = [np.array([lds[p * XR + xq(idx_Bp(h, L, r))] for L in range(64)]) for r in range(8)]
        ip = np.array([idx_Bp(h, L, 0) for L in range(64)])
        m2 = 2 * ((ip >> 1) & 1) + h
        t2 = [W[128 * m2], W[64 * m2], W[32 * m2], W[32 * m2 + 128]]
        for r in range(8):
            if not r & 1: bfly(X, r, r + 1, np.conj(t2[0]))
        for r in range(8):
            if not r & 2: bfly(X, r, r + 2, np.conj(mul_i(t2[1]) if r & 1 else t2[1]))
        for r in range(8):
            if r & 4: continue
            base = t2[3] if r & 1 else t2[2]
            bfly(X, r, r + 4, np.conj(mul_i(base) if r & 2 else base))
        loc = {}
        for r in range(8):
            for L in range(64): loc[xq(idx_Bp(h, L, r))] = X[r][L]
        X = [np.array([loc[xq(idx_B(h, L, r))] for L in range(64)]) for r in range(8)]
        m5 = 2 * (Lv & 15) + h
        w5, w6 = W[16 * m5], W[8 * m5]
        for r in range(8):
            if not r & 2: bfly(X, r, r + 2, np.conj(w5))
        for r in range(8):
            if not r & 4: bfly(X, r, r + 4, np.conj(mul_i(w6) if r & 2 else w6))
        for r in range(4): permlane(X[r], X[r + 4], 5)
        for r in range(8):
            if not r & 2: permlane(X[r], X[r + 2], 4)
        u = 2 * Lv + h
        w7, w8, w9a, w9b = W[4 * u], W[2 * u], W[u], W[u + 128]
        for r in range(8):
            if not r & 1: bfly(X, r, r + 1, np.conj(w7))
        for r in range(8):
            if not r & 2: bfly(X, r, r + 2, np.conj(mul_i(w8) if r & 1 else w8))
        for r in range(8):
            if r & 4: continue
            base = w9b if r & 1 else w9a
            bfly(X, r, r + 4, np.conj(mul_i(base) if r & 2 else base))
        for r in range(8):
            want = inv_ref[p][128 * r + u]
            err = max(err, np.abs(X[r] - want).max())
    print(f"inverse: max |kernel layout - oracle fft_inverse| = {err:.3e}")
    assert err < 1e-6
    print("qy layouts OK")


if __name__ == "__main__":
    main()
