"""Second pass of lds_layout_quad.py: also choose the lane order of phases B and C (the FFT bits a
phase keeps in lanes may sit on any lane bit), then the address weights."""
import itertools
import random
from lds_layout_quad import cost, lin

A = lambda h, L, r: 128 * r + 64 * h + L


def mk(lane_bits, reg_bits):
    # lane_bits[k] = FFT bit held by lane bit k; reg_bits[k] = FFT bit held by register bit k; h = b9
    def m(h, L, r):
        idx = 512 * h
        for k, b in enumerate(lane_bits):
            idx |= ((L >> k) & 1) << b
        for k, b in enumerate(reg_bits):
            idx |= ((r >> k) & 1) << b
        return idx
    return m


plain = lin([1 << i for i in range(10)])
B_lanes = [0, 1, 2, 3, 7, 8]
C_lanes = [0, 4, 5, 6, 7, 8]
best_b = min((cost(plain, A, True) + cost(plain, mk(p, [4, 5, 6]), False) + cost(plain, mk(p, [4, 5, 6]), True)
              + cost(plain, A, False), p) for p in itertools.permutations(B_lanes))
print("B", best_b)
Bm = mk(best_b[1], [4, 5, 6])
res = []
for p in itertools.permutations(C_lanes):
    if p.index(0) not in (4, 5):  # b0 on lane bit 4/5: last stage by v_permlane16/32_swap
        continue
    Cm = mk(p, [1, 2, 3])
    res.append((cost(plain, Bm, True) + cost(plain, Cm, False) + cost(plain, Cm, True) + cost(plain, Bm, False), p))
res.sort()
print("C", res[:3])
Cm = mk(res[0][1], [1, 2, 3])


def score(f):
    return (cost(f, A, True) + cost(f, Bm, False) + cost(f, Bm, True) + cost(f, Cm, False) +
            cost(f, Cm, True) + cost(f, Bm, False) + cost(f, Bm, True) + cost(f, A, False))


print("plain", score(plain))
random.seed(3)
cand = [0, 1, 2, 3, 4, 5, 8, 16, 17, 32, 33, 64]
out = []
for trial in range(30000):
    d = [random.choice(cand) if random.random() < 0.4 else 0 for _ in range(10)]
    w = [(1 << i) + d[i] for i in range(10)]
    f = lin(w)
    ad = [f(i) for i in range(1024)]
    if max(ad) >= 1088 or len(set(ad)) != 1024:
        continue
    out.append((score(f), max(ad), w))
out.sort()
print(out[:4])
f = lin(out[0][2])
for nm, m, wr in (("A wr", A, 1), ("B rd", Bm, 0), ("B wr", Bm, 1), ("C rd", Cm, 0), ("C wr", Cm, 1), ("A rd", A, 0)):
    print(nm, cost(f, m, wr))
