"""BASELINE config 3 on the GPU: 256-bit radix divided by a clear divisor (src/perf_test.rs:54 at
256 bits) plus the wide clear-operand scalar ops it rests on.

Parity bar: decrypted quotient / remainder equal floor division of the plaintexts (tfhe scalar div
semantics, 1344 / 5 = 268 at src/perf_test.rs:75), on seeded random 256-bit dividends with the
divisors SURVEY.md 8d names (5, a random u32, a random 128-bit value) and the edge cases (1, powers
of two, divisor wider than the dividend).  Encrypted divisors (FheUint / FheUint, SURVEY.md 8f
rank 1): same floor-division bar, and tfhe's division-by-zero convention (quotient all ones,
remainder = dividend)."""
import random

import pytest

from fhe_sign import (Context, FheUint8, FheUint32, FheUint64, FheUint128, FheUint256, generate_keys, multi_bit_params,
                      set_server_key, tuning)

pytestmark = pytest.mark.gpu
M256 = (1 << 256) - 1


@pytest.fixture(scope="module", params=["classic", "multibit"])
def keys(request):
    """classic (grouping 1) and multi-bit (grouping 2) blind rotation: the same decrypted results"""
    ck, sk = generate_keys(multi_bit_params() if request.param == "multibit" else None, seed=0xD1)
    ctx = Context(0)
    ctx.set_server_key(sk)
    set_server_key(ctx)
    yield ck, ctx
    set_server_key(None)
    ctx.close()


def test_perf_test_div_known_answer(keys):
    ck, _ = keys
    assert (FheUint32.try_encrypt(1344, ck) / 5).decrypt(ck) == 268  # src/perf_test.rs:54,75


@pytest.mark.parametrize("kind", ["5", "u32", "u128"])
def test_div256_by_clear(keys, kind):
    ck, _ = keys
    rng = random.Random(0xF11E51)
    a = rng.getrandbits(256) | 1 << 255
    d = {"5": 5, "u32": rng.getrandbits(32) | 1 << 31, "u128": rng.getrandbits(128) | 1 << 127}[kind]
    A = FheUint256.try_encrypt(a, ck)
    assert (A / d).decrypt(ck) == a // d
    if kind != "5":
        assert (A % d).decrypt(ck) == a % d


def test_div256_edge_divisors(keys):
    ck, _ = keys
    rng = random.Random(7)
    a = rng.getrandbits(256)
    A = FheUint256.try_encrypt(a, ck)
    assert (A / 1).decrypt(ck) == a
    assert (A / (1 << 77)).decrypt(ck) == a >> 77
    assert (A / (1 << 300)).decrypt(ck) == 0
    assert (A % (1 << 300)).decrypt(ck) == a
    small = FheUint256.try_encrypt(12345, ck)
    assert (small / ((1 << 200) + 3)).decrypt(ck) == 0
    with pytest.raises(Exception):
        A / 0


def test_wide_scalar_ops(keys):
    ck, _ = keys
    rng = random.Random(11)
    a, s = rng.getrandbits(128), rng.getrandbits(128) | 1 << 100
    A = FheUint128.try_encrypt(a, ck)
    m = (1 << 128) - 1
    assert (A & s).decrypt(ck) == a & s
    assert (A + s).decrypt(ck) == (a + s) & m
    assert (A * s).decrypt(ck) == (a * s) & m
    k = rng.getrandbits(128)
    assert A.scalar_mul_add(s, k).decrypt(ck) == (a * s + k) & m


@pytest.mark.parametrize("bits,cls", [(8, FheUint8), (32, FheUint32)])
def test_div_by_encrypted_random(keys, bits, cls):
    ck, _ = keys
    rng = random.Random(0xD1F + bits)
    m = (1 << bits) - 1
    cases = [(rng.getrandbits(bits), rng.getrandbits(rng.randint(1, bits)) or 1) for _ in range(3)]
    cases += [(rng.getrandbits(bits) >> 3, m), (m, 1), (m, m), (0, 7), (5, 9)]  # b > a, a = b, a = 0
    for a, b in cases:
        q, r = cls.try_encrypt(a, ck).div_rem(cls.try_encrypt(b, ck))
        assert (q.decrypt(ck), r.decrypt(ck)) == (a // b, a % b), (a, b)


def test_div_by_encrypted_zero(keys):
    ck, _ = keys
    A, Z = FheUint32.try_encrypt(123456789, ck), FheUint32.try_encrypt(0, ck)
    assert (A / Z).decrypt(ck) == (1 << 32) - 1
    assert (A % Z).decrypt(ck) == 123456789


def test_div_by_encrypted_operators(keys):
    ck, _ = keys
    rng = random.Random(64)
    a, b = rng.getrandbits(64), rng.getrandbits(40) | 1 << 39
    A, B = FheUint64.try_encrypt(a, ck), FheUint64.try_encrypt(b, ck)
    assert (A // B).decrypt(ck) == a // b
    assert (A % B).decrypt(ck) == a % b


def test_div256_by_encrypted(keys):
    ck, _ = keys
    rng = random.Random(256)
    a, b = rng.getrandbits(256) | 1 << 255, rng.getrandbits(128) | 1 << 127
    q, r = FheUint256.try_encrypt(a, ck).div_rem(FheUint256.try_encrypt(b, ck))
    assert (q.decrypt(ck), r.decrypt(ck)) == (a // b, a % b)


def test_public_scalar_recoding(keys):
    """Products with a public operand recode its base-4 digits to {-1, 0, 1, 2} (csrc/radix.cpp
    scalar_products: -x as 3 - x with a public -3): multipliers made of 3-digits (2^k - 1), mixed
    ones, wrap-around widths, multiply-add and the Granlund-Montgomery divisions that use them --
    equal to exact integer arithmetic."""
    ck, _ = keys
    rng = random.Random(0x5CA1)
    m = (1 << 128) - 1
    a = rng.getrandbits(128) | 1 << 127
    A = FheUint128.try_encrypt(a, ck)
    cases = [(1 << 128) - 1, (1 << 127) - 1, 0xFFFF_0000_FFFF_3333_3333_FFFF_0001_0003, 3, 0xF,
             rng.getrandbits(128)]
    for s in cases:
        got = [(A * s).decrypt(ck), A.scalar_mul_add(s, 0x3FFF).decrypt(ck)]
        want = [(a * s) & m, (a * s + 0x3FFF) & m]
        assert got == want, hex(s)
    for d in (3, 5, 0xFFFFFFFF, (1 << 64) - 59, (1 << 127) + 1):
        assert (A / d).decrypt(ck) == a // d, hex(d)
        assert (A % d).decrypt(ck) == a % d, hex(d)


@pytest.mark.parametrize("method", ["residue", "multiplier"])
def test_div256_residue_split(keys, method):
    with tuning(scalar_div_residue=1 if method == "residue" else 0):
        _div256_cases(keys)


def _div256_cases(keys):
    """Division by a public divisor, 256-bit dividends: the residue split a = d T + S (default for >= 64
    blocks; csrc/radix.cpp scalar_div_residue) and the multiplier method (tuning scalar_div_residue 0), on
    divisors across the split's range (3 up to 116 bits, even ones, 2^k +- 1) and dividends at the
    edges: quotient and remainder equal floor division."""
    ck, _ = keys
    rng = random.Random(0x5E51)
    for a, d in [(M256, 3), (rng.getrandbits(256), 10), (rng.getrandbits(256), (1 << 32) - 5),
                 (12345 * 1000003 + 77, 1000003), (rng.getrandbits(256), rng.getrandbits(64) | 1 << 63),
                 (rng.getrandbits(256), rng.getrandbits(116) | 1 << 115)]:
        A = FheUint256.try_encrypt(a, ck)
        assert (A / d).decrypt(ck) == a // d, (method, hex(d))
        assert (A % d).decrypt(ck) == a % d, (method, hex(d))
