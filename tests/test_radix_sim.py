"""Radix algorithms end to end on the CPU through the engine's simulating mode (Engine kSim,
fhe_host_sim_*): the operands are "encrypted" blocks whose plaintext the engine shadows on the host, so
every encrypted code path runs -- no trivial folding -- while each bootstrap is evaluated from its lookup
table and range-checked, with the degree and noise bookkeeping of the GPU runs.  Checked against exact
integer semantics (tfhe's for the radix ops: wrapping add/sub/mul, shift amounts mod the width, x / 0 =
all ones, x % 0 = x) and against oracle/ref_semantics.py for the BigUintFHE limbs (src/biguint.rs:120-265,
the compat mode's lost carries included).  The GPU tests run the same algorithms on ciphertexts."""
import ctypes as C
import os
import random

import pytest

import ref_semantics as R
from fhe_sign import _lib, tuning

COMPAT, FAST = 0, 1
DIVREM, MUL, ADD, SUB, SHR, LT, DIV_SCALAR, SHL, MUL_FULL, AND, MIN = range(11)
M32 = 1 << 32


def sim_radix(op, bits, a, b):
    w = (bits + 63) // 64
    A = (C.c_uint64 * w)(*[(a >> (64 * i)) & (2**64 - 1) for i in range(w)])
    B = (C.c_uint64 * w)(*[(b >> (64 * i)) & (2**64 - 1) for i in range(w)])
    out, out2 = (C.c_uint64 * (2 * w))(), (C.c_uint64 * w)()
    pbs, lev = C.c_uint64(), C.c_uint64()
    lib = _lib.load()
    rc = lib.fhe_host_sim_radix(op, bits, A, B, out, out2, C.byref(pbs), C.byref(lev))
    assert rc == 0, lib.fhe_last_error()
    return sum(out[i] << (64 * i) for i in range(2 * w)), sum(out2[i] << (64 * i) for i in range(w))


def sim_mul(a, b, mode, k=None):
    A = (C.c_uint32 * max(1, len(a)))(*a)
    B = (C.c_uint32 * max(1, len(b)))(*b)
    K = (C.c_uint32 * max(1, len(k)))(*k) if k else None
    cap = len(a) + len(b) + (len(k) if k else 0) + 2
    out, n = (C.c_uint32 * cap)(), C.c_size_t()
    kp = C.cast(K, C.POINTER(C.c_uint32)) if K is not None else None
    lib = _lib.load()
    rc = lib.fhe_host_sim_biguint_mul(A, len(a), B, len(b), kp, len(k) if k else 0, mode, out, cap, C.byref(n),
                                      None, None)
    assert rc == 0, lib.fhe_last_error()
    return list(out[: n.value])


def expect(op, bits, a, b):
    M = 1 << bits
    if op == DIVREM:
        return (a // b, a % b) if b else (M - 1, a)
    if op == SHR:
        return a >> (b % bits)
    if op == SHL:
        return (a << (b % bits)) % M
    return {MUL: lambda: a * b % M, ADD: lambda: (a + b) % M, SUB: lambda: (a - b) % M, LT: lambda: int(a < b),
            DIV_SCALAR: lambda: a // 0xC0FFEE01, MUL_FULL: lambda: a * b, AND: lambda: a & b,
            MIN: lambda: min(a, b)}[op]()


def operands(bits, rng, count):
    M = 1 << bits
    edge = [0, 1, 2, 3, M - 1, M - 2, M // 2, M // 2 - 1, (M - 1) // 3]
    out = [(x, y) for x in (0, 1, M - 1) for y in (0, 1, M - 1)]
    for _ in range(count):
        kind = rng.randrange(4)
        if kind == 0:
            out.append((rng.getrandbits(bits), rng.getrandbits(bits)))
        elif kind == 1:
            out.append((rng.choice(edge), rng.getrandbits(bits)))
        elif kind == 2:
            out.append((rng.getrandbits(bits), rng.getrandbits(max(1, bits // 3))))
        else:
            out.append((rng.choice(edge), rng.choice(edge)))
    return out


@pytest.mark.parametrize("bits", [2, 8, 16, 32, 64, 128, 256])
@pytest.mark.parametrize("op", [MUL, ADD, SUB, LT, DIV_SCALAR, MUL_FULL, AND, MIN])
def test_radix_ops_simulated(bits, op):
    rng = random.Random(1000 * op + bits)
    for a, b in operands(bits, rng, 6 if bits >= 128 else 14):
        got, _ = sim_radix(op, bits, a, b)
        assert got == expect(op, bits, a, b), (op, bits, hex(a), hex(b))


@pytest.mark.parametrize("bits", [2, 4, 8, 16, 32, 64, 256])
@pytest.mark.parametrize("op", [SHR, SHL])
def test_encrypted_shifts_simulated(bits, op):
    """The barrel shifters (4-way stages by amount blocks; one-block operands: the 2-way stage): every
    amount below the width at small widths, the amount's high bits ignored (mod the width)."""
    rng = random.Random(bits + 7 * op)
    M = 1 << bits
    amounts = range(bits) if bits <= 16 else [0, 1, 2, 3, 4, 7, 8, 31, bits // 2 + 1, bits - 1]
    for s in amounts:
        for a in (rng.getrandbits(bits), M - 1):
            for amt in (s, s + bits * rng.randrange(1, max(2, M // bits))):
                got, _ = sim_radix(op, bits, a, amt % M)
                assert got == expect(op, bits, a, amt % M), (op, bits, hex(a), amt)


@pytest.mark.parametrize("bits", [2, 8, 32, 64])
def test_encrypted_divrem_simulated(bits):
    rng = random.Random(bits)
    cases = operands(bits, rng, 10) + [(rng.getrandbits(bits), 0), (0, 0), ((1 << bits) - 1, 1)]
    for a, b in cases:
        assert sim_radix(DIVREM, bits, a, b) == expect(DIVREM, bits, a, b), (bits, hex(a), hex(b))


def test_encrypted_divrem_256_simulated():
    """The 256-bit / encrypted divisor (869 levels) on a few operand shapes, the zero divisor included."""
    rng = random.Random(256)
    M = 1 << 256
    for a, b in [(rng.getrandbits(256), rng.getrandbits(37) + 1), (M - 1, rng.getrandbits(256) | 1), (M - 1, 0),
                 (rng.getrandbits(255), (1 << 128) + 1)]:
        assert sim_radix(DIVREM, 256, a, b) == expect(DIVREM, 256, a, b)


@pytest.mark.parametrize("depth", [0, 7, 64])
def test_sliced_flushes_keep_results(depth):
    """The deferred graph launched in slices of `depth` levels (tuning flush_depth; default 64, 0 = only
    on demand): every slice is scheduled on its own, results unchanged -- the 256-bit division (660
    levels) and the compat 8 x 8 mul under small slices, and their schedules at the default depth within
    a fraction of a percent of the unsliced one."""
    rng = random.Random(64 + depth)
    with tuning(flush_depth=depth):
        a, b = rng.getrandbits(256), rng.getrandbits(130) | 1
        assert sim_radix(DIVREM, 256, a, b) == expect(DIVREM, 256, a, b)
        x, y = _limbs(rng, 8), _limbs(rng, 8)
        assert sim_mul(x, y, COMPAT) == R.biguint_mul(x, y)
    lib = _lib.load()
    p, lev = C.c_uint64(), C.c_uint64()
    with tuning(flush_depth=0):
        assert lib.fhe_host_radix_stats(DIVREM, 256, C.byref(p), C.byref(lev), None, 0) == 0
        p0, lev0 = p.value, lev.value
    assert lib.fhe_host_radix_stats(DIVREM, 256, C.byref(p), C.byref(lev), None, 0) == 0
    assert lev.value == lev0 and p.value <= p0 * 1.005, (p.value, lev.value, p0, lev0)


def _limbs(rng, n):
    special = [0, 1, M32 - 1, M32 - 2, M32 // 2, 0xFFFF0000, M32 - 16, 15, 16]
    return [rng.choice(special) if rng.random() < 0.4 else rng.getrandbits(32) for _ in range(n)]


@pytest.mark.parametrize("kara", [None, 6, 0])
def test_biguint_mul_simulated(kara):
    """BigUintFHE mul / mul-add on simulated limbs: compat (the reference's limbs, lost carries included)
    and fast (the true product) across limb shapes, with the Karatsuba split at its default threshold,
    recursing down to 6 blocks, and off (tuning kara_min / kara_compat_min)."""
    with tuning(**({} if kara is None else {"kara_min": kara, "kara_compat_min": kara})):
        _biguint_mul_cases(random.Random(5 if kara is None else 6 + kara))


def _biguint_mul_cases(rng):
    # 2 <= min <= 8: the carry-count chain; 1 or > 8 limbs (9 x 9, 12 x 4): the wave form; 0: zero
    shapes = [(1, 1), (2, 2), (1, 8), (8, 1), (3, 5), (8, 8), (9, 9), (12, 4), (0, 3), (3, 0)]
    for la, lb in shapes:
        a, b = _limbs(rng, la), _limbs(rng, lb)
        assert sim_mul(a, b, COMPAT) == R.biguint_mul(a, b), (la, lb)
        assert R.from_limbs(sim_mul(a, b, FAST)) == R.from_limbs(a) * R.from_limbs(b), (la, lb)
    full = [M32 - 1] * 8
    assert sim_mul(full, full, COMPAT) == R.biguint_mul(full, full)
    assert R.from_limbs(sim_mul(full, full, FAST)) == R.from_limbs(full) ** 2
    k = _limbs(rng, 8)
    a, b = _limbs(rng, 8), _limbs(rng, 8)
    assert sim_mul(a, b, COMPAT, k) == R.biguint_add(k, R.biguint_mul(a, b))
    assert R.from_limbs(sim_mul(a, b, FAST, k)) == R.from_limbs(a) * R.from_limbs(b) + R.from_limbs(k)


CALL_SITE = 0x200  # FHE_HOST_CALL_SITE


@pytest.mark.parametrize("mode", [COMPAT, FAST])
def test_call_site_mul_then_add_simulated(mode):
    """The reference's call site k_fhe + (e_fhe * privkey_fhe) as two ops (fhe_biguint_mul, then
    fhe_biguint_add with the product released unread): the add takes an exact product's block-product
    columns (BigUint::product_cols), the product's own normalization is dead and dropped -- same limbs
    as the reference's add of its mul, and the one-call mul-add's schedule (vector 0's 8 x 1 + 8 shape),
    not a second propagation.  Shapes without exact columns (compat 2..8 limbs: the chain) keep both ops."""
    rng = random.Random(11 + mode)
    for la, lb, lk in [(8, 1, 8), (1, 8, 8), (3, 1, 5), (1, 1, 1), (1, 1, 3), (8, 8, 8), (2, 3, 1)]:
        for _ in range(3):
            a, b, k = _limbs(rng, la), _limbs(rng, lb), _limbs(rng, lk)
            got = sim_mul(a, b, mode | CALL_SITE, k)
            if mode == COMPAT:
                assert got == R.biguint_add(k, R.biguint_mul(a, b)), (la, lb, lk)
            else:
                assert R.from_limbs(got) == R.from_limbs(a) * R.from_limbs(b) + R.from_limbs(k), (la, lb, lk)
    full = [M32 - 1] * 8
    assert sim_mul(full, [M32 - 1], mode | CALL_SITE, full) == R.biguint_add(full, R.biguint_mul(full, [M32 - 1]))
    lib = _lib.load()

    def stats(m):
        p, lev = C.c_uint64(), C.c_uint64()
        assert lib.fhe_host_biguint_mul_stats(8, 1, 8, m, C.byref(p), C.byref(lev), None, 0) == 0, lib.fhe_last_error()
        return p.value, lev.value

    assert stats(mode | CALL_SITE) == stats(mode)


DECRYPT_SUM = 0x400  # FHE_HOST_DECRYPT_SUM


@pytest.mark.parametrize("mode", [COMPAT, FAST])
def test_call_site_decrypt_reads_the_sums_columns(mode):
    """fhe_biguint_decrypt of a sum (the call site's `(k_fhe + e_fhe * privkey_fhe).to_biguint`) reads the
    sum's column form (BigUint::sum_cols) and launches only what that depends on (Engine::flush_for): the
    sim checks the columns' value against the digits' at that point, and the schedule is the product's
    alone -- the add's carry propagation stays pending (dead once the sum is released).  An add that
    took an exact product's columns (vector 0's 8 x 1 + 8) decrypts those columns compressed: the
    one-call column form's schedule (FHE_HOST_STATS_COLUMNS) plus at most one compression level."""
    rng = random.Random(23 + mode)
    for la, lb, lk in [(8, 8, 8), (8, 1, 8), (1, 8, 8), (2, 3, 1), (3, 1, 5), (1, 1, 3)]:
        a, b, k = _limbs(rng, la), _limbs(rng, lb), _limbs(rng, lk)
        got = sim_mul(a, b, mode | CALL_SITE | DECRYPT_SUM, k)
        assert R.from_limbs(got) == R.from_limbs(k) + R.from_limbs(sim_mul(a, b, mode)), (la, lb, lk)
    full = [M32 - 1] * 8
    for b in ([M32 - 1], full):
        got = sim_mul(full, b, mode | CALL_SITE | DECRYPT_SUM, full)
        assert R.from_limbs(got) == R.from_limbs(full) + R.from_limbs(sim_mul(full, b, mode))
    lib = _lib.load()

    def stats(la, lb, lk, m):
        p, lev = C.c_uint64(), C.c_uint64()
        assert lib.fhe_host_biguint_mul_stats(la, lb, lk, m, C.byref(p), C.byref(lev), None, 0) == 0, lib.fhe_last_error()
        return p.value, lev.value

    if mode == COMPAT:  # the chain's limbs: no product columns, the add is a plain sum
        lazy, full = stats(8, 8, 8, mode | CALL_SITE | DECRYPT_SUM), stats(8, 8, 8, mode | CALL_SITE)
        assert lazy == stats(8, 8, 0, mode)
        assert lazy[1] < full[1] and lazy[0] < full[0]
    lazy, full = stats(8, 1, 8, mode | CALL_SITE | DECRYPT_SUM), stats(8, 1, 8, mode | CALL_SITE)
    fused = stats(8, 1, 8, mode | 0x100)  # FHE_HOST_STATS_COLUMNS
    assert lazy[1] < full[1] and lazy[0] < full[0]
    assert lazy[1] <= fused[1] + 1 and lazy[0] <= fused[0] * 1.06


def sim_mul_add_columns(a, b, k, mode):
    A = (C.c_uint32 * max(1, len(a)))(*a)
    B = (C.c_uint32 * max(1, len(b)))(*b)
    K = (C.c_uint32 * max(1, len(k)))(*k)
    words, bits = (C.c_uint64 * 16)(), C.c_uint32()
    lib = _lib.load()
    rc = lib.fhe_host_sim_biguint_mul_add_columns(A, len(a), B, len(b), K, len(k), mode, words, 16, C.byref(bits),
                                                  None, None)
    assert rc == 0, lib.fhe_last_error()
    return sum(words[i] << (64 * i) for i in range(16)), bits.value


@pytest.mark.parametrize("mode", [COMPAT, FAST])
def test_mul_add_columns_simulated(mode):
    """k + a * b left in column form (the signer's FHE block without its final carry propagation): the
    columns' value, carries resolved on the host as the decryption does, equals the limbs' value of
    the normalized mul-add -- compat's lost carries included (8 x 8 limbs of all ones)."""
    rng = random.Random(11 + mode)
    shapes = [(8, 1, 8), (1, 8, 8), (8, 8, 8), (2, 3, 1), (8, 8, 0), (3, 2, 5)]
    for la, lb, lk in shapes:
        a, b, k = _limbs(rng, la), _limbs(rng, lb), _limbs(rng, lk)
        val, bits = sim_mul_add_columns(a, b, k, mode)
        want = sim_mul(a, b, mode, k) if lk else sim_mul(a, b, mode)
        assert val == R.from_limbs(want), (la, lb, lk)
        assert bits == 32 * (max(lk, la + lb) + 1)
    full = [M32 - 1] * 8
    val, _ = sim_mul_add_columns(full, full, [M32 - 1] * 8, mode)
    assert val == R.from_limbs(sim_mul(full, full, mode, [M32 - 1] * 8))


@pytest.mark.parametrize("bits", [8, 64, 290])
def test_scalar_mac_columns_simulated(bits):
    """The public-operand signer's column form (a * m + m with m public, recoded digits, no carry
    propagation): its value mod 2^bits."""
    rng = random.Random(bits)
    M = 1 << bits
    for a, m in operands(bits, rng, 6):
        got, _ = sim_radix(11, bits, a, m)
        assert got == (a * m + m) % M, (bits, hex(a), hex(m))


@pytest.mark.parametrize("lead", [0, 2, 6, 16, 256])
@pytest.mark.parametrize("bits", [16, 32, 64])
def test_encrypted_divrem_radix16_lead_simulated(lead, bits):
    with tuning(div_r16_lead=lead):
        _radix16_lead_cases(lead, bits)


def _radix16_lead_cases(lead, bits):
    """The leading radix-16 steps (tuning div_r16_lead = dividend blocks taken two at a time before the radix-4
    steps; 256 = every step) on divisors whose multiples c*d (c = 1..15) sit at the window boundaries
    4^w of the early steps, where the [c*d < 4^w] flags (d's high blocks zero and the exact low multiple
    c*(d mod 4^L) below 4^w) decide the candidate set."""
    rng = random.Random(bits * 31 + int(lead))
    M = 1 << bits
    divisors = {1, 2, 3, 5, 15, 16, 17, M - 1, M // 2, M // 2 + 1}
    for w in (1, 2, 3, 4, 6):
        for c in (1, 3, 5, 7, 11, 15):
            for delta in (-1, 0, 1):
                d = (4 ** w) // c + delta
                if 0 < d < M:
                    divisors.add(d)
    divisors = sorted(divisors)
    rng.shuffle(divisors)
    for d in divisors[:14]:
        for a in (M - 1, rng.getrandbits(bits), d * rng.randrange(1, 16) + rng.randrange(d)):
            a %= M
            assert sim_radix(DIVREM, bits, a, d) == expect(DIVREM, bits, a, d), (lead, bits, hex(a), hex(d))


DIVREM_CLEAR, DIVREM_CLEAR_MIXED = 12, 13


@pytest.mark.parametrize("residue", [0, 1, -1])
@pytest.mark.parametrize("bits", [32, 128, 256])
def test_scalar_divrem_simulated(residue, bits):
    """a / d and a % d for PUBLIC divisors (radix_scalar_div / _rem): the multiplier method (tuning
    scalar_div_residue 0), the residue split a = d T + S wherever it is valid (1) and the size rule (-1,
    the default), on divisors from 3 up to beyond the residue split's range, odd and even, 2^k +- 1."""
    with tuning(scalar_div_residue=residue):
        _scalar_divrem_cases(residue, bits)


def _scalar_divrem_cases(residue, bits):
    rng = random.Random(bits * 7 + (residue if residue >= 0 else 5))
    M = 1 << bits
    divisors = [3, 5, 6, 7, 10, 12, 255, 257, 1000003, 0xC0FFEE01, (1 << 31) - 1, (1 << 32) - 5,
                rng.getrandbits(20) | 1, rng.getrandbits(40) | 3, rng.getrandbits(bits // 2) | 1]
    for d in divisors:
        d %= M
        if d < 2:
            continue
        for a in (M - 1, 0, d - 1, d, rng.getrandbits(bits), d * rng.getrandbits(max(1, bits - d.bit_length()))):
            a %= M
            assert sim_radix(DIVREM_CLEAR, bits, a, d) == (a // d, a % d), (residue, bits, hex(a), hex(d))
            # a's odd blocks trivial (public constants inside the dividend: the exact columns' excess)
            assert sim_radix(DIVREM_CLEAR_MIXED, bits, a, d) == (a // d, a % d), (residue, bits, hex(a), hex(d))


@pytest.mark.parametrize("bits", [512, 4096])
def test_radix_ops_max_width_simulated(bits):
    """The widest radix (FHE_RADIX_MAX_BITS = 4096, 2048 blocks) and 512 bits: add / sub / lt / and /
    min / encrypted shr and a public-divisor division (the residue split at these widths), every
    bootstrap simulated; 512-bit products too."""
    rng = random.Random(bits)
    M = 1 << bits
    ops = [ADD, SUB, LT, AND, MIN, SHR] + ([MUL, DIV_SCALAR] if bits == 512 else [])
    for op in ops:
        for a, b in [(M - 1, M - 1), (rng.getrandbits(bits), rng.getrandbits(bits)), (0, M - 1)]:
            if op == SHR:
                b = rng.randrange(bits)
            got, _ = sim_radix(op, bits, a, b)
            assert got == expect(op, bits, a, b), (op, bits)


# ---- the compat chain's g (csrc/compat_chain.cpp compat_chain_g) on hand-built prefix columns
def _chain_g_expect(v):
    k = sum(x << (2 * m) for m, x in enumerate(v)) % M32
    near = k >= M32 - 16
    return 15 - (k % 16 if near else 0)


def _chain_g_record(v):
    """31 block values of a prefix whose column sums are v (v[0] <= 3, v[m] <= 6)"""
    rec = [v[0]]
    for x in v[1:]:
        a = min(x, 3)
        rec += [a, x - a]
    return rec


def _unresolve(v, rng, moves):
    """move value between columns without changing K: +4 at column m, -1 at m + 1 (and back)"""
    v = list(v)
    for _ in range(moves):
        m = rng.randrange(1, 15)
        if rng.random() < 0.5:
            if v[m] + 4 <= 6 and v[m + 1] >= 1:
                v[m] += 4
                v[m + 1] -= 1
        elif v[m] >= 4 and v[m + 1] + 1 <= 6:
            v[m] -= 4
            v[m + 1] += 1
    return v


def test_chain_g_carry_aware_near():
    """near = [K mod 2^32 >= 2^32 - 16] with carries moving through blocks that resolve to 3 (ADVICE r5:
    v_1 >= 4, v_2 = 6, v_3.. = 3 resolves to blocks 3..15 = 0; v_3.. = 2 and runs of 6 resolve to 3)"""
    rng = random.Random(0xC4A1)
    cases = [
        [3, 4, 6] + [3] * 13,            # carry through block 2 into 3: blocks 3..15 resolve to 0 -> near 0
        [3, 4, 6] + [2] * 13,            # ... resolve to 3 -> near 1
        [1, 4, 6, 6, 6, 2] + [3] * 10,   # a run of 6s carrying, ended by a 2
        [2, 4, 6, 6, 6, 6] + [2] * 10,
        [0, 0, 3] + [3] * 13,            # plain all-3
        [3, 3, 3] + [3] * 13,
        [3, 4, 2] + [3] * 13,            # carry absorbed at block 2
        [3, 5, 6] + [6] * 13,            # carries out of the top: K mod 2^32 small
        [3, 6, 6] + [6] * 12 + [2],
    ]
    # random representations of values at the boundary (K mod 2^32 in [2^32 - 40, 2^32 + 24), and the
    # same above 2^32)
    for base in (0, M32):
        for t in range(-40, 24):
            kk = (base + M32 + t) % (2 * M32)
            canon = [(kk >> (2 * m)) & 3 for m in range(16)]
            if kk >= M32:  # 2^32 sits above column 15: put it there as 4 extra units of column 15
                canon[15] += 4
            for _ in range(4):
                v = _unresolve(canon, rng, rng.randrange(0, 40))
                if sum(x << (2 * m) for m, x in enumerate(v)) == kk and max(v[1:]) <= 6 and v[0] <= 3:
                    cases.append(v)
    for _ in range(200):
        cases.append([rng.randrange(4)] + [rng.choice([2, 3, 3, 3, 6, rng.randrange(7)]) for _ in range(15)])
    vals = bytes(b for v in cases for b in _chain_g_record(v))
    g = (C.c_uint32 * len(cases))()
    pbs, lev = C.c_uint64(), C.c_uint64()
    lib = _lib.load()
    rc = lib.fhe_host_sim_chain_g((C.c_uint8 * len(vals)).from_buffer_copy(vals), len(cases), g, C.byref(pbs),
                                  C.byref(lev))
    assert rc == 0, lib.fhe_last_error()
    assert lev.value == 5
    assert pbs.value == 33 * len(cases)
    bad = [(v, g[i], _chain_g_expect(v)) for i, v in enumerate(cases) if g[i] != _chain_g_expect(v)]
    assert not bad, bad[:4]
    assert sum(_chain_g_expect(v) != 15 for v in cases) >= 40  # the boundary cases do reach near = 1
