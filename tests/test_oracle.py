"""The CPU oracle itself: FFT / negacyclic product / PBS correctness (test infrastructure).

The oracle restates tfhe 0.10.0's PBS (published algorithm; crate absent).  Its
known-answer checks are mathematical: the FFT must realise the exact negacyclic product up to
rounding, and PBS(Enc(m), f) must decrypt to f(m) for every m.
"""
import numpy as np
import pytest

import oracle

rng = np.random.default_rng(1234)


def negacyclic(a, b):
    n = len(a)
    c = [0] * n
    for i in range(n):
        if a[i] == 0:
            continue
        for j in range(n):
            k = i + j
            if k < n:
                c[k] += a[i] * b[j]
            else:
                c[k - n] -= a[i] * b[j]
    return c


def test_fft_roundtrip_exact_scaling():
    x = rng.standard_normal(1024) + 1j * rng.standard_normal(1024)
    y = oracle.fft_inverse(oracle.fft_forward(x)) / 1024
    assert np.max(np.abs(y - x)) < 1e-12


def test_fft_matches_numpy_dft():
    x = rng.standard_normal(1024) + 1j * rng.standard_normal(1024)
    f = oracle.fft_forward(x)
    # DIF output is bit-reversed; twiddles are exp(+2 pi i k / 1024)
    rev = np.array([int(format(i, "010b")[::-1], 2) for i in range(1024)])
    ref = np.fft.ifft(x) * 1024
    assert np.max(np.abs(f[rev] - ref)) < 1e-9


def test_twisted_forward_equals_twist_then_dif():
    """The blind rotation's digit transform (negacyclic split with zeta twiddles, no separate twist)
    computes the same values, in the same bit-reversed order, as twist by psi^j + the DIF transform
    the bootstrapping key is converted with (different rounding, same mathematics)."""
    x = rng.integers(-2**22, 2**22, 1024) + 1j * rng.integers(-2**22, 2**22, 1024)
    psi = np.exp(1j * np.pi * np.arange(1024) / 2048)
    a = oracle.fft_forward_twisted(x)
    b = oracle.fft_forward(x * psi)
    assert np.max(np.abs(a - b)) < 1e-9 * np.max(np.abs(b))


def test_f64_to_torus():
    assert oracle.f64_to_torus(0.0) == 0
    assert oracle.f64_to_torus(-0.0) == 0
    assert oracle.f64_to_torus(2.5) == 2          # half-even
    assert oracle.f64_to_torus(3.5) == 4
    assert oracle.f64_to_torus(-1.0) == 2**64 - 1
    assert oracle.f64_to_torus(2.0**64) == 0
    assert oracle.f64_to_torus(2.0**70 + 2.0**20) == 2**20
    assert oracle.f64_to_torus(-(2.0**63)) == 2**63
    assert oracle.f64_to_torus(1e30) == int(1e30) % 2**64


@pytest.fixture(scope="module")
def okeys():
    return oracle.OracleKeys(99)


def test_pbs_identity_and_square_all_messages(okeys):
    r = okeys.rng(5)
    f = [(m * m + 3) % 16 for m in range(16)]
    lut = okeys.make_lut(f)
    ident = okeys.make_lut(list(range(16)))
    for m in range(16):
        ct = okeys.encrypt(r, m)
        assert okeys.decrypt(okeys.pbs(ct, lut)) == f[m]
    for m in (0, 7, 15):
        out = okeys.pbs(okeys.encrypt(r, m), ident)
        assert okeys.decrypt(out) == m
        noise = (okeys.phase(out) - m * okeys.delta() + 2**63) % 2**64 - 2**63
        assert abs(noise) < 2**54  # fresh PBS noise far below delta/2 = 2^58


def test_simd_paths_bit_identical(okeys):
    """The SIMD loops of the oracle's classic blind rotation and keyswitch (what bench.py's
    cpu_baseline times: AVX2, and AVX-512 where the CPU has it) against its scalar restatement
    (fho_set_simd(0)): the same ciphertexts give identical words at every level the CPU supports,
    through every LUT-rotation and monomial pattern a random batch reaches."""
    lib = oracle.load()
    top = lib.fho_simd()
    if top == 0:
        pytest.skip("oracle built without AVX2/FMA")
    r = okeys.rng(11)
    cts = np.stack([okeys.encrypt(r, m % 16) for m in range(12)])
    luts = np.stack([okeys.make_lut([(m * 5 + k) % 16 for m in range(16)]) for k in range(3)])
    idx = (np.arange(12) % 3).astype(np.uint32)
    res = {}
    try:
        for level in range(top + 1):
            lib.fho_set_simd(level)
            assert lib.fho_simd() == level
            res[level] = okeys.pbs_batch(cts, luts, idx, 4), okeys.keyswitch_batch(cts, 4)
    finally:
        lib.fho_set_simd(-1)
    assert lib.fho_simd() == top
    for level in range(1, top + 1):
        assert np.array_equal(res[level][1], res[0][1]), f"keyswitch, level {level}"
        assert np.array_equal(res[level][0], res[0][0]), f"PBS, level {level}"
    assert [okeys.decrypt(res[top][0][i]) for i in range(12)] == [((i % 16) * 5 + i % 3) % 16 for i in range(12)]


def test_keyswitch_preserves_message(okeys):
    r = okeys.rng(6)
    n = okeys.params.n
    for m in (0, 5, 11):
        ct = okeys.encrypt(r, m)
        small = okeys.keyswitch(ct)
        phase = (int(small[n]) - int(np.dot(small[:n].astype(object), okeys.lwe_sk.astype(object)))) % 2**64
        err = (phase - m * okeys.delta() + 2**63) % 2**64 - 2**63
        assert abs(err) < 2**57


def test_noise_budget_at_radix_limit_oracle(okeys):
    """CPU twin of tests/test_pbs_gpu.py::test_noise_budget_at_radix_limit on the oracle: the
    carry prefix's largest PBS input, 4 s0 + 2 s1 + s2 + c of fresh bootstrap outputs (22 of the
    radix layer's 25-variance budget), keyswitched and modulus-switched, keeps > 8 sigma of margin
    against the half step (64 in the 4096-domain)."""
    rs = np.random.default_rng(6)
    N = 160
    s = rs.integers(0, 3, size=(3, N))
    c = rs.integers(0, 2, size=N)
    r = okeys.rng(78)
    fresh = np.stack([okeys.encrypt(r, int(v)) for v in np.concatenate([s.ravel(), c])])
    ident = okeys.make_lut(list(range(16)))[None, :]
    unit = okeys.pbs_batch(fresh, ident, np.zeros(len(fresh), np.uint32)).astype(np.uint64)
    with np.errstate(over="ignore"):
        comb = (np.uint64(4) * unit[:N] + np.uint64(2) * unit[N:2 * N] + unit[2 * N:3 * N] + unit[3 * N:]).astype(np.uint64)
    m = 4 * s[0] + 2 * s[1] + s[2] + c
    n = okeys.params.n
    sk = okeys.lwe_sk.astype(object)
    errs = []
    for i in range(N):
        small = okeys.keyswitch(comb[i])
        ms = [((int(w) + (1 << 51)) >> 52) % 4096 for w in small[: n + 1]]
        phase = (ms[n] - sum(a * b for a, b in zip(ms[:n], sk))) % 4096
        errs.append((phase - 128 * int(m[i]) + 2048) % 4096 - 2048)
    errs = np.array(errs, dtype=np.float64)
    assert np.abs(errs).max() < 64
    print(f"modulus-switched sigma at 22 units: {errs.std():.2f} (half step 64)")
    assert errs.std() * 8 < 64, f"modulus-switched sigma {errs.std():.2f}"


def test_noise_failure_sample_oracle_10k(okeys):
    """CPU mirror of tests/test_noise_gpu.py on the oracle: 10^4 PBS inputs at the radix
    layer's noise limit -- 5000 of the carry prefix's 22-unit shape 4 s0 + 2 s1 + s2 + c and 5000 of
    the 25-unit shape 4 s + 3 c -- built from a pool of 384 oracle bootstrap outputs (distinct index
    tuples; tuples share pool blocks, so the samples are correlated, not independent), keyswitched
    (batched) and modulus-switched: the blind rotation's input error in the 4096-domain must stay
    below the half step (64) for every one of them -- zero decode failures -- and its sigma must
    match the modulus-switch model sqrt((n/2 + 1) / 12) (the dominant term) within 15 %."""
    rs = np.random.default_rng(0x10_000)
    ns, nc = 256, 128
    sv, cv = rs.integers(0, 3, ns), rs.integers(0, 2, nc)
    r = okeys.rng(79)
    fresh = np.stack([okeys.encrypt(r, int(v)) for v in np.concatenate([sv, cv])])
    ident = okeys.make_lut(list(range(16)))[None, :]
    unit = okeys.pbs_batch(fresh, ident, np.zeros(len(fresh), np.uint32)).astype(np.uint64)
    us, uc = unit[:ns], unit[ns:]
    K = 5000
    ia = np.stack([rs.choice(ns, 3, replace=False) for _ in range(K)])
    ic = rs.integers(0, nc, K)
    ib = rs.integers(0, ns, K)
    jc = rs.integers(0, nc, K)
    with np.errstate(over="ignore"):
        comb_a = np.uint64(4) * us[ia[:, 0]] + np.uint64(2) * us[ia[:, 1]] + us[ia[:, 2]] + uc[ic]
        comb_b = np.uint64(4) * us[ib] + np.uint64(3) * uc[jc]
    m = np.concatenate([4 * sv[ia[:, 0]] + 2 * sv[ia[:, 1]] + sv[ia[:, 2]] + cv[ic], 4 * sv[ib] + 3 * cv[jc]])
    assert m.max() <= 15
    small = okeys.keyswitch_batch(np.concatenate([comb_a, comb_b]))
    n = okeys.params.n
    ms = ((small.astype(object) + (1 << 51)) >> 52) % 4096
    ms = ms.astype(np.int64)
    phase = (ms[:, n] - ms[:, :n] @ okeys.lwe_sk.astype(np.int64)) % 4096
    err = (phase - 128 * m + 2048) % 4096 - 2048
    fails = int((np.abs(err) >= 64).sum())
    model = np.sqrt((n / 2 + 1) / 12)
    print(f"\noracle: {2 * K} inputs at 22/25 units, {fails} failures; MS-domain sigma 22u {err[:K].std():.2f}, "
          f"25u {err[K:].std():.2f} (modulus-switch model {model:.2f}; half step 64); max |err| {np.abs(err).max()}")
    assert fails == 0
    for e in (err[:K], err[K:]):
        assert abs(e.std() / model - 1) < 0.15


def _exact(x: float) -> int:
    return int(x)  # every operand below is an integer-valued double (|x| >= 2^53 or built from an int)


def _bal(v: int, m: int) -> int:
    v %= m
    return v - m if v >= m // 2 else v


@pytest.mark.parametrize("ylog", [97, 90.5])
def test_unreduced_accumulator_error_bound(ylog):
    """the f64 accumulator is reduced mod 2^64 only on every second update, so the next
    step's digit input can carry |y| <= 2^97 (worst case; ~2^90.5 typical).  Since round 3 the
    classic CMUX is factored (oracle fho_blind_rotate) and takes the digits of acc itself, as the
    multi-bit path always did: model an accumulator coefficient after an unreduced update,
    a = red(a0) + ya (one rounding), and its digit (oracle fho_tor_digit, base 2^23), and compare with
    exact integer torus arithmetic: the digit must stay balanced (|d| <= 2^22) and be off the exact
    digit by at most 2^5 digit units (2^46 of the torus) worst case -- the bound restated at
    tfhe_oracle.c:fho_blind_rotate, far below the 2^58 decode half-step; then the reducing update
    red(a + y2) must be exact mod 2^64 and land in [-2^63, 2^63]."""
    lib = oracle.load()
    rs = np.random.default_rng(7)
    T = 1 << 64
    worst = 0
    for _ in range(4000):
        a0 = float(int(rs.integers(-(1 << 62), 1 << 62, dtype=np.int64)) * 2)
        sa = rs.choice([-1.0, 1.0])
        ya = float(round(sa * float(2.0 ** ylog) * (1 - rs.random() * 2**-20)))
        a = a0 + ya  # unreduced update: one rounding
        d = lib.fho_tor_digit(a, 23)  # the factored CMUX's digit of acc itself
        assert abs(d) <= 2**22 and d == int(d)
        v_true = _exact(a0) + _exact(ya)
        d_true = _bal((v_true + (1 << 40)) >> 41, 1 << 23)  # round(v / 2^41) mod 2^23, balanced
        err = abs(_bal(int(d) - d_true, 1 << 23))
        worst = max(worst, err)
        # the following (reducing) update: exact mod 2^64 and back in range
        y2 = float(round(sa * 2.0 ** ylog * rs.random()))
        s = a + y2
        r = lib.fho_tor_red(s)
        assert abs(r) <= 2.0**63 and (_exact(r) - _exact(s)) % T == 0
    bound = 2**5 if ylog >= 97 else 2**0
    print(f"\n|y| ~ 2^{ylog}: worst digit error {worst} digit units (bound {bound}; 1 unit = 2^41 of the torus)")
    assert worst <= bound
