"""Integer-level model of the compat BigUintFHE mul as a carry-count chain (csrc/biguint.cpp
compat_chain), checked against oracle/ref_semantics.py:biguint_mul (src/biguint.rs:194-265).

The reference's step (i, j) adds P = a_i b_j into the 96-bit window of limbs idx = i + j .. idx + 2
and drops the carry out of its top.  Per limb l the touches come in step order with roles
  BOT (idx = l):     add lo(P), no carry in, crossing forwarded to l + 1
  MID (idx = l - 1): add hi(P) + carry in, crossing forwarded (dropped if l is the top limb)
  TOP (idx = l - 2): carry in only, crossing dropped.
With K(t) = the known addends so far and k(t) = the carries in so far (k <= 15 when min(la, lb) <= 8),
crossings so far C(t) = floor((K + k) / 2^32) = H + beta, H = floor(K / 2^32),
beta = [K mod 2^32 + k >= 2^32] = [k - g - 1 >= 0], g = 15 - near * (K mod 16),
near = [K mod 2^32 >= 2^32 - 16].  Carries into l + 1 up to step s telescope over l's touches:
  k_{l+1}(s) = H_l(u) + beta_l(u) - sum_{TOP touches w <= s} (beta_l(w) - beta_l(prev w)),
u = l's last touch at or before s (a TOP touch adds nothing to K, so H cancels there).
The final limb is (K_l(last) + k_l(final)) mod 2^32.  Only the beta's form a serial chain, one
lookup per limb.

usage: python3 tools/compat_chain_sim.py [trials]
"""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import ref_semantics as R  # noqa: E402

M = 1 << 32


def touches(la, lb):
    """per limb: list of (step index, i, j, role) in reference step order"""
    L = la + lb
    T = [[] for _ in range(L)]
    s = 0
    for i in range(la):
        for j in range(lb):
            idx = i + j
            T[idx].append((s, i, j, "BOT"))
            T[idx + 1].append((s, i, j, "MID"))
            if idx + 2 < L:
                T[idx + 2].append((s, i, j, "TOP"))
            s += 1
    return T


def compat_chain(a, b):
    la, lb = len(a), len(b)
    if not la or not lb:
        return []
    assert min(la, lb) <= 8
    L = la + lb
    T = touches(la, lb)
    P = {(i, j): a[i] * b[j] for i in range(la) for j in range(lb)}
    # prefix quantities per limb and touch (off the chain: products and prefix sums only)
    K = [[0] * len(T[l]) for l in range(L)]
    for l in range(L):
        acc = 0
        for n, (s, i, j, role) in enumerate(T[l]):
            if role == "BOT":
                acc += P[i, j] % M
            elif role == "MID":
                acc += P[i, j] // M
            K[l][n] = acc
    H = [[x // M for x in K[l]] for l in range(L)]
    g = [[15 - ((x % M) % 16 if (x % M) >= M - 16 else 0) for x in K[l]] for l in range(L)]
    beta = [[0] * len(T[l]) for l in range(L)]
    kfinal = [0] * L
    for l in range(L):
        prev = T[l - 1] if l else []

        def k_at(s):
            # carries into l up to step s, from limb l - 1's betas
            u = max((m for m, t in enumerate(prev) if t[0] <= s), default=None)
            if u is None:
                return 0
            k = H[l - 1][u] + beta[l - 1][u]
            for m, t in enumerate(prev):
                if t[0] <= s and t[3] == "TOP":
                    k -= beta[l - 1][m] - (beta[l - 1][m - 1] if m else 0)
            return k

        for n, (s, i, j, role) in enumerate(T[l]):
            k = k_at(s)
            assert 0 <= k <= 15, (l, n, k)
            v = k - g[l][n] - 1
            assert -16 <= v <= 14
            beta[l][n] = 1 if v >= 0 else 0
            # cross-check against the definition
            assert beta[l][n] == ((K[l][n] % M) + k >= M)
        kfinal[l] = k_at(1 << 30)
    return [(K[l][-1] + kfinal[l]) % M if T[l] else 0 for l in range(L)]


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    rng = random.Random(7)
    special = [0, 1, M - 1, M - 2, M // 2, 0xFFFF0000, 0x0000FFFF, M - 16, M - 17, 15, 16]
    cases = 0
    for t in range(trials):
        la, lb = rng.randint(1, 8), rng.randint(1, 8)
        if t % 7 == 0:
            lb = rng.randint(1, 12)  # one side above 8 limbs
        mode = t % 4
        if mode == 0:
            a = [rng.getrandbits(32) for _ in range(la)]
            b = [rng.getrandbits(32) for _ in range(lb)]
        elif mode == 1:
            a = [rng.choice(special) for _ in range(la)]
            b = [rng.choice(special) for _ in range(lb)]
        elif mode == 2:
            a = [M - 1] * la
            b = [M - 1] * lb
        else:
            a = [rng.choice((M - 1, rng.getrandbits(32))) for _ in range(la)]
            b = [rng.choice((M - 1, 1, rng.getrandbits(32))) for _ in range(lb)]
        if min(la, lb) > 8:
            continue
        want = R.biguint_mul(a, b)
        got = compat_chain(a, b)
        assert got == want, (a, b, got, want)
        cases += 1
    print(f"compat chain model == reference limb loop on {cases} cases")


if __name__ == "__main__":
    main()
