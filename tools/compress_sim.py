"""Simulator of csrc/radix.cpp:compress_columns (block degrees and noise only) and of the tail
pass-through variant (h1): bootstraps and rounds for product column sets.  usage: python3 tools/compress_sim.py"""
# simulator of csrc/radix.cpp:compress_columns (degrees/noise only), and variants
import sys
KMAXT, KMAXN = 6, 25

def product_cols(na, nb, nblocks):
    cols = [[] for _ in range(nblocks)]
    for p in range(na):
        for q in range(nb):
            if p + q < nblocks:
                cols[p+q].append((3, 1))
            if p + q + 1 < nblocks:
                cols[p+q+1].append((2, 1))
    return cols

def groups_current(c):
    c = sorted(c, key=lambda x: -x[0])
    s, end = 0, len(c)
    out = []
    while s < end:
        g = []; deg = noi = 0
        while s < end and len(g) < KMAXT:
            mn = c[end-1][0]
            slots = min(KMAXT - len(g) - 1, end - s - 1)
            if deg + c[s][0] + slots * mn <= 15 and noi + c[s][1] <= KMAXN:
                pick = c[s]; s += 1
            elif deg + mn <= 15 and noi + c[end-1][1] <= KMAXN:
                end -= 1; pick = c[end]
            else:
                break
            g.append(pick); deg += pick[0]; noi += pick[1]
        out.append(g)
    return out

def compress(cols, lim0=7, lim=6, maxb=3, variant="current"):
    cols = [list(c) for c in cols]
    n = len(cols)
    pbs = rounds = 0
    while True:
        nxt = [[] for _ in range(n)]
        in_deg = in_noise = in_cnt = 0
        anyc = False
        for k in range(n):
            c = cols[k]
            L = lim0 if k == 0 else lim
            deg = sum(x[0] for x in c); noi = sum(x[1] for x in c)
            if deg + in_deg <= L and len(c) + in_cnt <= maxb and noi + in_noise <= KMAXN - 1:
                nxt[k] += c
                in_deg = in_noise = in_cnt = 0
                continue
            anyc = True
            out_deg = out_noise = out_cnt = 0
            if variant == "current":
                gs = groups_current(c)
                keep = []
            else:
                gs, keep = variant(c, in_deg, in_cnt, L, maxb)
            nxt[k] += keep
            for g in gs:
                d = sum(x[0] for x in g)
                if len(g) == 1 and d <= 3 and g[0][1] <= 1:
                    nxt[k].append(g[0]); continue
                pbs += 1
                nxt[k].append((min(3, d), 1))
                if d >= 4 and k + 1 < n:
                    pbs += 1
                    nxt[k+1].append((min(d >> 2, 3), 1))
                    out_deg += min(d >> 2, 3); out_noise += 1; out_cnt += 1
            in_deg, in_noise, in_cnt = out_deg, out_noise, out_cnt
        if not anyc:
            return pbs, rounds, cols
        rounds += 1
        cols = nxt

if __name__ == "__main__":
    for (na, nb, nbk) in [(16, 16, 32), (128, 128, 128), (128, 16, 144)]:
        p, r, _ = compress(product_cols(na, nb, nbk))
        print(na, nb, nbk, "current:", p, "PBS", r, "rounds")

def make_h1(thresh_deg, thresh_cnt):
    def v(c, in_deg, in_cnt, L, maxb):
        gs = groups_current(c)
        keep = []
        out = []
        for g in gs:
            d = sum(x[0] for x in g)
            if d <= thresh_deg and len(g) <= thresh_cnt and all(x[1] <= 1 for x in g):
                keep += g
            else:
                out.append(g)
        # must still make progress: if nothing compressed, compress everything
        if not out:
            return gs, []
        return out, keep
    return v

def h2(c, in_deg, in_cnt, L, maxb):
    # compress only enough: largest-first full groups until the remaining pass-through + produced lo's
    # + incoming fit the final bound, else keep going
    c = sorted(c, key=lambda x: -x[0])
    gs = groups_current(c)
    # try leaving the smallest groups out while the column would still be "final" after this round
    best = (gs, [])
    for drop in range(1, len(gs)):
        kept = [x for g in gs[len(gs)-drop:] for x in g]
        out = gs[:len(gs)-drop]
        deg = sum(x[0] for x in kept) + sum(min(3, sum(y[0] for y in g)) for g in out) + in_deg
        cnt = len(kept) + len(out) + in_cnt
        if deg <= L and cnt <= maxb:
            best = (out, kept)
    return best

if __name__ == "__main__":
    shapes = [(16, 16, 32), (128, 128, 256), (128, 16, 144)]
    for (na, nb, nbk) in shapes:
        base = compress(product_cols(na, nb, nbk))
        res = [("cur", base[0], base[1])]
        for td, tc in [(3, 1), (5, 2), (6, 2), (8, 3), (9, 3), (11, 4)]:
            p, r, _ = compress(product_cols(na, nb, nbk), variant=make_h1(td, tc))
            res.append((f"h1({td},{tc})", p, r))
        p, r, _ = compress(product_cols(na, nb, nbk), variant=h2)
        res.append(("h2", p, r))
        print(na, nb, nbk, res)
