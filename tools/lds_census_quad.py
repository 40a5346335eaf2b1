#!/usr/bin/env python3
"""LDS cycle census of one CMUX of the 4-wave blind rotation (br_quad.hip, classic), per wave.
Layout "r3" is the round-3 kernel (stage 9 across lane pairs, b0 = L0, b8 = L2); "s9" has b0 on
lane bit 2 and b8 on L0, with stage 9 in registers after a register-bit-2 <-> lane-bit-2 transpose
(two zeta reads instead of eight, the zeta table swizzled, the digit swap on a lane-linear map).  The rotation sites of the
round-2 kernel are gone with the factored CMUX.

Every LDS instruction of the loop with its per-lane byte addresses, costed by the gfx950 rules of
MI355X_MICROARCH.md's LDS table: lane groups per instruction, one LDS-array cycle per group when
conflict-free, +1 per extra distinct address on a bank within a group; stores also pay their
data transfer (2 cycles per source dword per wave-instruction: b64 6, b128 13), so a store costs
max(transfer, array cycles).  Prints per site the array cycles, the conflict-free minimum and the
charged cycles, then the totals.  usage: python3 tools/lds_census_quad.py [r3|s9]
"""
import sys

QX_SZ, QTW_SZ, QZ_LDS = 1093, 512 + 16, 546
QL_W, QL_Z = 2 * QX_SZ, 2 * QX_SZ + QTW_SZ
QZ_ONE, QZ_MINUS_I = 544, 545
WQ = [1, 2, 4, 8, 16, 32, 66, 132, 274, 541]  # br_quad.hip


def fq(i):
    return sum(w for k, w in enumerate(WQ) if i >> k & 1)


def tpos(k):
    return k + (k >> 5)


def groups(kind):
    if kind in ("r64", "r32"):
        return [list(range(0, 32)), list(range(32, 64))]
    if kind == "r128":
        g = [[0, 1, 2, 3, 12, 13, 14, 15] + list(range(20, 28)), [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
        return g + [[l + 32 for l in x] for x in g]
    if kind == "w64":
        return [list(range(16 * k, 16 * k + 16)) for k in range(4)]
    if kind == "w128":
        return [list(range(8 * k, 8 * k + 8)) for k in range(8)]
    raise ValueError(kind)


def cycles(kind, addr):
    """addr[lane] = byte address; returns (array cycles, conflict-free array cycles, charged)"""
    size = {"r32": 4, "r64": 8, "r128": 16, "w64": 8, "w128": 16}[kind]
    nbanks = 64 if kind.startswith("r") and kind != "r32" else 32
    arr = 0
    for g in groups(kind):
        banks = {}
        for lane in g:
            a = addr[lane]
            for d in range(size // 4):
                b = (a // 4 + d) % nbanks
                banks.setdefault(b, set()).add(a // 4 + d)
        arr += max(len(v) for v in banks.values())
    base = len(groups(kind))
    xfer = {"w64": 6, "w128": 13}.get(kind, 0)
    return arr, base, max(arr, xfer)


def main():
    lay = sys.argv[1] if len(sys.argv) > 1 else "r3"
    s9 = lay == "s9"
    # zeta-table swizzle of the S9 kernel (br_quad.hip zsw)
    zs = (lambda k: k ^ (((k >> 4) & 1) << 2) if k >= 32 else k) if s9 else (lambda k: k)
    sites = []  # (name, kind, [addr per lane]) per wave-instruction; averaged over the 4 waves
    for w in range(4):
        p, h = w >> 1, w & 1
        region = p * QX_SZ * 16
        L = list(range(64))
        t = [64 * h + l for l in L]
        bit = lambda l, k: (l >> k) & 1
        b8 = (lambda l: bit(l, 0)) if s9 else (lambda l: bit(l, 2))
        b0 = (lambda l: bit(l, 2)) if s9 else (lambda l: bit(l, 0))
        u = [16 * b8(l) + 8 * bit(l, 1) + 4 * bit(l, 5) + 2 * bit(l, 4) + bit(l, 3) for l in L]
        lowB = [8 * bit(l, 5) + 4 * bit(l, 4) + 2 * bit(l, 3) + b0(l) for l in L]
        B3 = [4 * h + 2 * b8(l) + bit(l, 1) for l in L]
        B6 = [32 * h + uu for uu in u]
        z9 = [288 + 32 * h + uu for uu in u]
        bA = [fq(tt) for tt in t]
        bB = [fq(512 * h + 256 * b8(l) + 128 * bit(l, 1) + lowB[l]) for l in L]
        if s9:  # digit swap: lane bits -> idx bits 5..0, registers -> 8..6
            bC = [fq(512 * h + l) for l in L]
            regC = [fq(64 * r) for r in range(8)]
        else:
            bC = [fq(512 * h + 16 * u[l] + bit(l, 0)) for l in L]
            regC = [fq(2 * r) for r in range(8)]
        cpl = lambda idx: [16 * i for i in idx]
        S = lambda name, kind, ad: sites.append((name, kind, ad))
        for r in range(8):
            S("A->B write", "w128", [region + 16 * (b + fq(128 * r)) for b in bA])
        for r in range(8):
            S("A->B read", "r128", [region + 16 * (b + fq(16 * r)) for b in bB])
        for off in (0, 8, 16, 24):
            S("zeta B", "r128", cpl([QL_Z + zs(off + b) for b in B3]))
        for off in (32, 96, 160, 224):
            S("zeta C", "r128", cpl([QL_Z + zs(off + b) for b in B6]))
        if s9:
            for b2 in range(2):
                S("zeta 9", "r128", cpl([QL_Z + zs(z9[l] + 128 * bit(l, 2) + 64 * b2) for l in L]))
        else:
            for r2 in range(4):
                ia = [z9[l] + 64 * r2 if l & 1 else QZ_ONE for l in L]
                ib = [ia[l] if l & 1 else QZ_MINUS_I for l in L]
                S("zeta 9", "r128", cpl([QL_Z + i for i in ia]))
                S("zeta 9", "r128", cpl([QL_Z + i for i in ib]))
        for r in range(8):
            S("digit swap write", "w128", [region + 16 * (b + regC[r]) for b in bC])
        oreg = (1 - p) * QX_SZ * 16
        for r in range(8):
            S("digit swap read", "r128", [oreg + 16 * (b + regC[r]) for b in bC])
        # inverse twiddles: q_dit<K> reads sw[lb] (and sw[lb + 132] for K = 2)
        def tw(name, lane_part):
            for K, lp in zip((0, 1, 2), lane_part):
                lb = [tpos(x) for x in lp]
                S(name, "r128", cpl([QL_W + x for x in lb]))
                if K == 2:
                    S(name, "r128", cpl([QL_W + x + 132 for x in lb]))
        tw("twiddle C", ([256 * b0(l) for l in L], [128 * b0(l) for l in L], [64 * b0(l) for l in L]))
        tw("twiddle B", ([32 * x for x in lowB], [16 * x for x in lowB], [8 * x for x in lowB]))
        for r in range(8):
            S("B->A write", "w128", [region + 16 * (b + fq(16 * r)) for b in bB])
        for r in range(8):
            S("B->A read", "r128", [region + 16 * (b + fq(128 * r)) for b in bA])
        tw("twiddle A", ([4 * tt for tt in t], [2 * tt for tt in t], list(t)))
    agg = {}
    for name, kind, ad in sites:
        arr, base, ch = cycles(kind, ad)
        e = agg.setdefault(name, [kind, 0, 0, 0, 0])
        e[1] += 1
        e[2] += arr
        e[3] += base
        e[4] += ch
    tot = [0, 0, 0]
    print(f"{'site':18s} {'kind':5s} {'instr':>5s} {'array':>7s} {'min':>7s} {'charged':>8s}   (per wave, layout {lay})")
    for name, (kind, n, arr, base, ch) in agg.items():
        print(f"{name:18s} {kind:5s} {n / 4:5.0f} {arr / 4:7.1f} {base / 4:7.1f} {ch / 4:8.1f}")
        tot[0] += arr / 4
        tot[1] += base / 4
        tot[2] += ch / 4
    print(f"{'total':18s} {'':5s} {'':5s} {tot[0]:7.1f} {tot[1]:7.1f} {tot[2]:8.1f}")


if __name__ == "__main__":
    main()
