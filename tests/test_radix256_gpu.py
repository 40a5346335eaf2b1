"""north_star's 256-bit op set on the HIP path: sub, encrypted shift (both directions), encrypted and
clear `&` on FheUint256 operands, classic and multi-bit blind rotation.

The reference applies these ops at 32 bits (`>>` by an encrypted amount at src/perf_test.rs:36, `& 1`
at :48, shift amount mod the width at src/biguint.rs:494-498); north_star asks for them on 256-bit
encrypted integers.  Parity bar: decrypted value == the exact tfhe wrapping semantics restated in
oracle/ref_semantics.py (u_sub / u_shr / u_shl / u_and), every value of every case.

All cases of a test are issued before the first host read, so the deferred engine schedules them as
one graph (the sixteen barrel shifters share their levels)."""
import random

import pytest

import ref_semantics as R
from fhe_sign import Context, FheUint256, generate_keys, multi_bit_params, set_server_key, stats

pytestmark = pytest.mark.gpu
W = 256
M = (1 << W) - 1
SHIFTS = (0, 1, 31, 32, 127, 255, 256, 300)  # 256 and 300: amount taken mod the width


@pytest.fixture(scope="module", params=["classic", "multibit"])
def keys(request):
    ck, sk = generate_keys(multi_bit_params() if request.param == "multibit" else None, seed=0x256)
    ctx = Context(0)
    ctx.set_server_key(sk)
    set_server_key(ctx)
    yield ck, ctx
    set_server_key(None)
    ctx.close()


def test_sub256_wrap(keys):
    ck, _ = keys
    rng = random.Random(0x5B)
    x, y = rng.getrandbits(W), rng.getrandbits(W)
    cases = [(x, y), (y, x), (x, x), (0, 1), (0, M), (M, M), (1 << 255, (1 << 255) + 1), (M, 0)]
    enc = {v: FheUint256.try_encrypt(v, ck) for v in {v for c in cases for v in c}}
    outs = [(a, b, enc[a] - enc[b]) for a, b in cases]
    for a, b, o in outs:
        assert o.decrypt(ck) == R.u_sub(a, b, W), (hex(a), hex(b))


@pytest.mark.parametrize("direction", ["shr", "shl"])
def test_shift256_by_encrypted_amount(keys, direction):
    ck, ctx = keys
    rng = random.Random(0x5F + (direction == "shl"))
    x = rng.getrandbits(W) | 1 << 255 | 1
    X = FheUint256.try_encrypt(x, ck)
    ref = R.u_shr if direction == "shr" else R.u_shl
    p0, _ = stats(ctx)
    outs = [(s, (X >> FheUint256.try_encrypt(s, ck)) if direction == "shr" else (X << FheUint256.try_encrypt(s, ck)))
            for s in SHIFTS]
    for s, o in outs:
        assert o.decrypt(ck) == ref(x, s, W), (direction, s)
    assert stats(ctx)[0] > p0  # bootstrapped on the device, not folded on the host


def test_shift256_amount_high_bits_ignored(keys):
    """an amount with bits above log2(256) set (2^200 + 3) shifts by 3: tfhe's mod-width rule"""
    ck, _ = keys
    x = random.Random(9).getrandbits(W)
    X = FheUint256.try_encrypt(x, ck)
    s = (1 << 200) + 3
    S = FheUint256.try_encrypt(s, ck)
    r, l_ = X >> S, X << S
    assert r.decrypt(ck) == R.u_shr(x, s, W)
    assert l_.decrypt(ck) == R.u_shl(x, s, W)


def test_and256_encrypted_and_clear(keys):
    ck, _ = keys
    rng = random.Random(0xA4D)
    x, y = rng.getrandbits(W), rng.getrandbits(W)
    X, Y = FheUint256.try_encrypt(x, ck), FheUint256.try_encrypt(y, ck)
    Z, F = FheUint256.try_encrypt(0, ck), FheUint256.try_encrypt(M, ck)
    clears = [1, 0, M, rng.getrandbits(W), (1 << 255) | 1, 0xFFFFFFFF]
    enc = [(X & Y, x & y), (X & Z, 0), (X & F, x), (F & F, M), (X & X, x)]
    clr = [(X & c, R.u_and(x, c, W)) for c in clears]
    for o, want in enc + clr:
        assert o.decrypt(ck) == want


def test_sub_shift_and_chain256(keys):
    """the ops composed as a caller chains them: ((a - b) >> Enc(s)) & c, then << Enc(t)"""
    ck, _ = keys
    rng = random.Random(0xC4A1)
    a, b, c = rng.getrandbits(W), rng.getrandbits(W), rng.getrandbits(W)
    s, t = rng.randrange(W), rng.randrange(W)
    A, B = FheUint256.try_encrypt(a, ck), FheUint256.try_encrypt(b, ck)
    S, T = FheUint256.try_encrypt(s, ck), FheUint256.try_encrypt(t, ck)
    out = (((A - B) >> S) & c) << T
    want = R.u_shl(R.u_and(R.u_shr(R.u_sub(a, b, W), s, W), c, W), t, W)
    assert out.decrypt(ck) == want


def test_max_width_ops(keys):
    """The widest radix the ABI accepts (FHE_RADIX_MAX_BITS = 4096 bits, 2048 blocks per operand):
    add, sub, lt, min and encrypted shr, exact tfhe semantics on random and all-ones operands (division
    at this width is a 1.6M-bootstrap triangle: its algorithm is checked at 512 bits in
    test_radix_sim.py and at 256 bits in test_div_gpu.py)."""
    from fhe_sign import FheUint
    ck, _ = keys
    B = 4096
    MB = (1 << B) - 1
    rng = random.Random(0x4096)
    x, y, s = rng.getrandbits(B), rng.getrandbits(B), rng.randrange(B)
    X, Y, F = (FheUint.try_encrypt(v, ck, bits=B) for v in (x, y, MB))
    S = FheUint.try_encrypt(s, ck, bits=B)
    assert (X + Y).decrypt(ck) == (x + y) & MB
    assert (F + F).decrypt(ck) == (2 * MB) & MB
    assert (X - Y).decrypt(ck) == (x - y) & MB
    assert X.lt(Y).decrypt(ck) == int(x < y) and F.lt(X).decrypt(ck) == 0
    assert X.min(Y).decrypt(ck) == min(x, y)
    assert (X >> S).decrypt(ck) == x >> s
