"""LDS exchange layout for the 4-wave blind rotate (k_blind_rotate_quad): one linear address map f
over the 10 FFT index bits, scored with the gfx950 b128 lane-group model of lds_layout_search.py.
Thread (h, L), register r (8 per lane) hold FFT index:
  A: 128 r + 64 h + L                       (regs b9 b8 b7)
  B: 512 h + 256 L5 + 128 L4 + 16 r + L&15  (regs b6 b5 b4)
  C: 512 h + 32 (L>>1) ... = 512 h + 16 (L>>1) + 2 r + (L&1)   (regs b3 b2 b1; b0 = L0)
Exchanges: A<->B (cross-wave), B<->C (wave-private, inside the b9 = h half)."""
import random
from lds_layout_search import RG128, WG128, cyc

A = lambda h, L, r: 128 * r + 64 * h + L
B = lambda h, L, r: 512 * h + 256 * ((L >> 5) & 1) + 128 * ((L >> 4) & 1) + 16 * r + (L & 15)
C = lambda h, L, r: 512 * h + 16 * (L >> 1) + 2 * r + (L & 1)


def cost(f, m, write):
    g, ns = (WG128, 8) if write else (RG128, 16)
    tot = 0
    for h in range(2):
        for r in range(8):
            tot += cyc([f(m(h, L, r)) for L in range(64)], g, ns)
    return tot / 16 / (8 if write else 4)


def lin(w):
    return lambda idx: sum(w[i] for i in range(10) if idx >> i & 1)


def score(f):
    return (cost(f, A, True) + cost(f, B, False) + cost(f, B, True) + cost(f, C, False) +
            cost(f, C, True) + cost(f, B, False) + cost(f, B, True) + cost(f, A, False))


if __name__ == "__main__":
    print("plain", score(lin([1 << i for i in range(10)])))
    random.seed(2)
    cand = [0, 1, 2, 3, 4, 5, 8, 16, 17, 32, 33, 64]
    res = []
    for trial in range(60000):
        d = [random.choice(cand) if random.random() < 0.5 else 0 for _ in range(10)]
        w = [(1 << i) + d[i] for i in range(10)]
        f = lin(w)
        ad = [f(i) for i in range(1024)]
        if max(ad) >= 1088 or len(set(ad)) != 1024:
            continue
        res.append((score(f), max(ad), w))
    res.sort()
    for r in res[:5]:
        print(r)
    w = res[0][2]
    f = lin(w)
    for nm, m, wr in (("A wr", A, 1), ("B rd", B, 0), ("B wr", B, 1), ("C rd", C, 0), ("C wr", C, 1), ("A rd", A, 0)):
        print(nm, cost(f, m, wr))
