"""GPU radix layer (FheUint ops) and BigUintFHE against the reference semantics.

Parity bar: decrypted values equal the reference's (tfhe wrapping semantics; BigUintFHE limb
loop of src/biguint.rs:120-265 incl. the :247-249 wrap) on the reference's known answers and on
seeded random inputs.  Ciphertext bytes vs tfhe-rs: parity unpinned."""
import json
import os
import random

import pytest

import ref_semantics as R
from conftest import ROOT
from fhe_sign import (COMPAT, FAST, BigUintFHE, Context, FheUint8, FheUint32, FheUint64, generate_keys,
                      multi_bit_params, set_server_key, stats)

pytestmark = pytest.mark.gpu
G = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module", params=["classic", "multibit"])
def keys(request):
    """classic (grouping 1) and multi-bit (grouping 2) blind rotation: the same decrypted results"""
    ck, sk = generate_keys(multi_bit_params() if request.param == "multibit" else None, seed=0xB16)
    ctx = Context(0)
    ctx.set_server_key(sk)
    set_server_key(ctx)
    yield ck, ctx
    set_server_key(None)
    ctx.close()


def test_fheuint_known_answers(keys):
    ck, _ = keys
    for c in json.load(open(os.path.join(G, "known_answers.json")))["fheuint"]:
        T = FheUint64 if c["bits"] == 64 else FheUint32
        a = T.try_encrypt(c["a"], ck)
        if c["op"] == "add_split":  # extract_upper_bits / extract_lower_bits (src/biguint.rs:108-117)
            s = a + T.try_encrypt(c["b"], ck)
            hi = FheUint32.cast_from(s >> 32)
            lo = FheUint32.cast_from(s & 0xFFFFFFFF)
            assert (hi.decrypt(ck), lo.decrypt(ck)) == (c["hi"], c["lo"]), c["test"]
        elif c["op"] == "add_shr_and":  # &sum >> 32, &sum & mask on the same width
            s = a + T.try_encrypt(c["b"], ck)
            assert ((s >> 32).decrypt(ck), (s & 0xFFFFFFFF).decrypt(ck)) == (c["hi"], c["lo"]), c["test"]
        elif c["op"] == "scalar_mul":
            assert (a * c["b"]).decrypt(ck) == c["value"], c["test"]
        elif c["op"] == "scalar_add":
            assert (a + c["b"]).decrypt(ck) == c["value"], c["test"]
        elif c["op"] == "add":
            assert (a + T.try_encrypt(c["b"], ck)).decrypt(ck) == c["value"], c["test"]
        elif c["op"] == "mul":
            assert (a * T.try_encrypt(c["b"], ck)).decrypt(ck) == c["value"], c["test"]
        elif c["op"] == "scalar_div":
            assert (a / c["b"]).decrypt(ck) == c["value"], c["test"]
        elif c["op"] == "perf_chain":  # src/perf_test.rs:36-63
            b = T.try_encrypt(c["b"], ck)
            shifted = a >> b
            casted = shifted.cast_into(FheUint8)
            m = casted.min(FheUint8.try_encrypt(c["c"], ck))
            assert (m & 1).decrypt(ck) == c["value"], c["test"]


def test_fheuint32_random_ops(keys):
    ck, _ = keys
    rng = random.Random(7)
    M = 1 << 32
    for _ in range(3):
        x, y = rng.getrandbits(32), rng.getrandbits(32)
        a, b = FheUint32.try_encrypt(x, ck), FheUint32.try_encrypt(y, ck)
        assert (a + b).decrypt(ck) == (x + y) % M
        assert (a - b).decrypt(ck) == (x - y) % M
        assert (a * b).decrypt(ck) == (x * y) % M
        s = rng.randrange(64)
        assert (a >> s).decrypt(ck) == x >> (s % 32)
        assert (a << s).decrypt(ck) == (x << (s % 32)) % M
        m = rng.getrandbits(32)
        assert (a & m).decrypt(ck) == x & m
        d = rng.randrange(1, 1 << 20)
        assert (a / d).decrypt(ck) == x // d
        assert (a % d).decrypt(ck) == x % d
        assert a.min(b).decrypt(ck) == min(x, y)
        assert a.max(b).decrypt(ck) == max(x, y)
        assert a.lt(b).decrypt(ck) == int(x < y)
        sh = rng.randrange(32)
        assert (a >> FheUint32.try_encrypt(sh, ck)).decrypt(ck) == x >> sh


def test_fheuint_edge_cases(keys):
    ck, _ = keys
    M = 1 << 32
    z, f = FheUint32.try_encrypt(0, ck), FheUint32.try_encrypt(M - 1, ck)
    assert (f + f).decrypt(ck) == (2 * M - 2) % M
    assert (f * f).decrypt(ck) == 1
    assert (z - f).decrypt(ck) == 1
    assert z.lt(z).decrypt(ck) == 0 and z.lt(f).decrypt(ck) == 1 and f.lt(z).decrypt(ck) == 0
    assert (f / 3).decrypt(ck) == (M - 1) // 3
    assert (f >> 32).decrypt(ck) == M - 1  # shift mod width (src/biguint.rs:494-498)
    with pytest.raises(Exception):
        f / 0
    e8 = FheUint8.try_encrypt(255, ck)
    assert (e8 + FheUint8.try_encrypt(1, ck)).decrypt(ck) == 0
    assert FheUint64.cast_from(f).decrypt(ck) == M - 1
    assert FheUint8.cast_from(f).decrypt(ck) == 255


def _big(ck, limbs):
    return BigUintFHE.new(R.from_limbs(limbs), ck)


def test_biguint_known_answers(keys):
    ck, _ = keys
    for c in json.load(open(os.path.join(G, "known_answers.json")))["biguint"]:
        a = BigUintFHE.new(c["a"], ck)
        if c["op"] == "roundtrip":
            assert a.to_biguint(ck) == c["value"]
            continue
        b = BigUintFHE.new(c["b"], ck)
        out = a + b if c["op"] == "add" else a * b
        if "limbs" in c:
            assert out.decrypt_limbs(ck) == c["limbs"], c["test"]
        else:
            assert out.to_biguint(ck) == c["value"], c["test"]


def test_biguint_add_256_compat_and_fast(keys):
    ck, _ = keys
    g = json.load(open(os.path.join(G, "biguint_vectors.json")))
    for v in g["add"][:3]:
        a, b = _big(ck, v["a"]), _big(ck, v["b"])
        assert a.add(b, COMPAT).decrypt_limbs(ck) == v["out"]
        assert a.add(b, FAST).decrypt_limbs(ck) == v["out"]
    for v in g["edge"]:
        a, b = _big(ck, v["a"]), _big(ck, v["b"])
        out = (a.add(b) if v["op"] == "add" else a.mul(b)).decrypt_limbs(ck)
        assert out == v["out"]


def test_biguint_mul_256_compat(keys):
    """config 2: 8x8-limb BigUintFHE mul, exact reference limb loop (src/biguint.rs:214-254)."""
    ck, ctx = keys
    g = json.load(open(os.path.join(G, "biguint_vectors.json")))
    v = g["mul"][0]
    p0, l0 = stats(ctx)
    out = _big(ck, v["a"]).mul(_big(ck, v["b"]), COMPAT)
    assert out.decrypt_limbs(ck) == v["out"]
    p1, l1 = stats(ctx)
    assert p1 > p0 and l1 > l0


def test_biguint_mul_256_config2_breadth(keys):
    """config 2 breadth on the HIP path: every committed seeded 8x8 pair, BIP-340 vector 1's e*d'
    and the all-ones (F7) pair, each in compat (the reference's limbs, src/biguint.rs:194-265, lost
    carries included) and fast (true product) mode.  All 20 products are issued before the first
    host read, so the deferred engine runs them as ONE schedule (throughput-bound, not 20 x the
    latency floor)."""
    ck, _ = keys
    g = json.load(open(os.path.join(G, "biguint_vectors.json")))
    v1 = json.load(open(os.path.join(G, "sign_vectors.json")))["vectors"][1]
    q = g["quirk_mul"][0]
    pairs = [(v["a"], v["b"], v["out"]) for v in g["mul"]] + [(v1["e"], v1["d"], v1["prod"]),
                                                              (q["a"], q["b"], q["out"])]
    assert len(pairs) == 10
    outs = []
    for a, b, want in pairs:
        A, B = _big(ck, a), _big(ck, b)
        outs.append((A.mul(B, COMPAT), A.mul(B, FAST), a, b, want))
    for i, (oc, of, a, b, want) in enumerate(outs):
        assert oc.decrypt_limbs(ck) == want, i
        assert R.from_limbs(of.decrypt_limbs(ck)) == R.from_limbs(a) * R.from_limbs(b), i
    assert outs[-1][0].decrypt_limbs(ck) == q["out"] != q["true_product"]


def test_biguint_mul_quirk_compat_vs_fast(keys):
    """F7: (2^256-1)^2 -- compat reproduces the reference's lost carry, fast gives the true product."""
    ck, _ = keys
    q = json.load(open(os.path.join(G, "biguint_vectors.json")))["quirk_mul"][0]
    a, b = _big(ck, q["a"]), _big(ck, q["b"])
    assert a.mul(b, COMPAT).decrypt_limbs(ck) == q["out"]
    assert a.mul(b, FAST).decrypt_limbs(ck) == q["true_product"]


def test_sign_fhe_with_k0_vector0_limb_flow(keys):
    """config 4 FHE block (src/schnorr.rs:272-275) on BIP-340 vector 0: e*d' (8x1 limbs) then k + ."""
    ck, _ = keys
    v = json.load(open(os.path.join(G, "sign_vectors.json")))["vectors"][0]
    e, d, k = _big(ck, v["e"]), _big(ck, v["d"]), _big(ck, v["k"])
    prod = e * d.clone()
    assert prod.decrypt_limbs(ck) == v["prod"]
    s = k + prod
    assert s.decrypt_limbs(ck) == v["sum"]
    assert s.to_biguint(ck) % R.N == int(v["s"], 16)


def test_sum_decrypted_from_its_columns(keys):
    """fhe_biguint_decrypt of a sum reads the sum's column form and launches only what that depends on
    (Engine::flush_for): the sum's own carry propagation stays pending -- run when the sum is used again
    (its digits, a further add), dropped as dead before the next recording once the sum is released."""
    ck, ctx = keys
    v = json.load(open(os.path.join(G, "sign_vectors.json")))["vectors"][0]
    e, d, k = _big(ck, v["e"]), _big(ck, v["d"]), _big(ck, v["k"])
    s = k + e * d  # exact 8 x 1 product: the add takes its columns (compressed ones decrypted)
    assert s.decrypt_limbs(ck) == v["sum"]
    assert s.to_biguint(ck) % R.N == int(v["s"], 16)
    t = s + k  # the pending propagation of s feeds a further add
    assert t.decrypt_limbs(ck) == R.biguint_add(v["sum"], v["k"])
    assert [x.decrypt(ck) for x in s.digits] == v["sum"]  # the digits themselves (a full flush)
    rng = random.Random(0x5C01)
    al, bl = R.to_u32_digits(rng.getrandbits(256)), R.to_u32_digits(rng.getrandbits(224))
    a, b = _big(ck, al), _big(ck, bl)
    p0, _ = stats(ctx)
    assert (a + b).decrypt_limbs(ck) == R.biguint_add(al, bl)
    assert stats(ctx)[0] == p0  # the operands' own blocks: nothing launched
    # released after the decryption: its propagation never runs -- the next op launches its own
    # bootstraps only (as many as the same op on a clean engine)
    counts = []
    for _ in range(2):
        x = a + b
        assert x.decrypt_limbs(ck) == R.biguint_add(al, bl)
        del x
        p1, _ = stats(ctx)
        assert (a * d).decrypt_limbs(ck) == R.biguint_mul(al, v["d"])
        counts.append(stats(ctx)[0] - p1)
    p2, _ = stats(ctx)
    assert (a * d).decrypt_limbs(ck) == R.biguint_mul(al, v["d"])
    assert counts == [stats(ctx)[0] - p2] * 2


def test_biguint_mul_add_equals_mul_then_add(keys):
    """fhe_biguint_mul_add (the signer's FHE block k + e*d' in one schedule) gives the limbs of
    add(k, mul(a, b)) of src/biguint.rs in both modes: exact 8x1 (k enters the product columns), the
    8x8 compat product with the F7 lost carry (lazy last waves feed the add), fast, zero operands."""
    ck, _ = keys
    v = json.load(open(os.path.join(G, "sign_vectors.json")))["vectors"][0]
    e, d, k = _big(ck, v["e"]), _big(ck, v["d"]), _big(ck, v["k"])
    assert e.mul_add(d, k).decrypt_limbs(ck) == v["sum"]
    q = json.load(open(os.path.join(G, "biguint_vectors.json")))["quirk_mul"][0]
    rng = random.Random(0x5EED)
    kl = R.to_u32_digits(rng.getrandbits(256))
    a, b, kk = _big(ck, q["a"]), _big(ck, q["b"]), _big(ck, kl)
    assert a.mul_add(b, kk, COMPAT).decrypt_limbs(ck) == R.biguint_add(kl, R.biguint_mul(q["a"], q["b"]))
    got = a.mul_add(b, kk, FAST).decrypt_limbs(ck)
    assert R.from_limbs(got) == R.from_limbs(kl) + R.from_limbs(q["a"]) * R.from_limbs(q["b"])
    assert len(got) == max(len(kl), len(q["a"]) + len(q["b"])) + 1
    zero = BigUintFHE.new(0, ck)
    assert a.mul_add(zero, kk).decrypt_limbs(ck) == kl
    assert a.mul_add(b, zero, COMPAT).decrypt_limbs(ck) == R.biguint_mul(q["a"], q["b"])


def test_biguint_mul_add_columns_value(keys):
    """The signer's column form (fhe_biguint_mul_add_columns + fhe_columns_decrypt: k + a*b without its
    final carry propagation, carries resolved by the decryption) gives the value of mul_add's limbs:
    the 8x1 signer shape, the 8x8 compat product with the F7 lost carry, fast, a zero addend."""
    ck, _ = keys
    v = json.load(open(os.path.join(G, "sign_vectors.json")))["vectors"][0]
    e, d, k = _big(ck, v["e"]), _big(ck, v["d"]), _big(ck, v["k"])
    assert e.mul_add_value(d, k, ck) == R.from_limbs(v["sum"])
    q = json.load(open(os.path.join(G, "biguint_vectors.json")))["quirk_mul"][0]
    rng = random.Random(0xC015)
    kl = R.to_u32_digits(rng.getrandbits(256))
    a, b, kk = _big(ck, q["a"]), _big(ck, q["b"]), _big(ck, kl)
    assert a.mul_add_value(b, kk, ck, COMPAT) == R.from_limbs(R.biguint_add(kl, R.biguint_mul(q["a"], q["b"])))
    want = R.from_limbs(kl) + R.from_limbs(q["a"]) * R.from_limbs(q["b"])
    assert a.mul_add_value(b, kk, ck, FAST) == want
    zero = BigUintFHE.new(0, ck)
    assert a.mul_add_value(b, zero, ck, COMPAT) == R.from_limbs(R.biguint_mul(q["a"], q["b"]))


def test_deferred_graph_lifetimes_and_raw_pbs(keys):
    """The engine defers bootstraps until a host read (csrc/radix.h Engine): operands and results
    dropped before that read keep what the pending graph still needs, raw fhe_pbs_batch calls in
    between (same stream, same workspace) neither see nor disturb pending work, and a graph built
    over several calls runs as one schedule with every value right."""
    import numpy as np
    ck, ctx = keys
    rng = random.Random(0xDEF)
    xs = [rng.getrandbits(32) for _ in range(6)]
    a = [FheUint32.try_encrypt(x, ck) for x in xs]
    s01 = a[0] + a[1]
    p23 = a[2] * a[3]
    dropped = a[4] * a[5]  # never read
    del dropped
    del a[4:]
    q = (s01 * p23) + a[0]
    del a[1:]  # operands of pending bootstraps
    inc = ctx.lut([(m + 1) % 16 for m in range(16)])
    cts = np.stack([ck.encrypt_block(m) for m in range(8)])
    raw = ctx.pbs(cts, inc)  # raw path while the radix graph is still pending
    assert [ck.decrypt_block(c) for c in raw] == [(m + 1) % 16 for m in range(8)]
    m = 2**32
    assert q.decrypt(ck) == (((xs[0] + xs[1]) % m) * ((xs[2] * xs[3]) % m) + xs[0]) % m
    assert s01.decrypt(ck) == (xs[0] + xs[1]) % m
    assert p23.decrypt(ck) == (xs[2] * xs[3]) % m


def test_biguint_compat_uneven_limbs(keys):
    """Compat mul / mul_add on uneven limb counts (2x3, 5x2, 3x4, 4x4 with all-ones limbs that make
    the reference drop carries): the lazy window waves, the 2-limb last windows and the top-run
    carry prefix against oracle/ref_semantics.py's replay of src/biguint.rs:194-265."""
    ck, _ = keys
    rng = random.Random(0xC0DA)
    for la, lb in ((2, 3), (5, 2), (3, 4), (4, 4)):
        for trial in range(2):
            if trial == 0:
                al = [rng.getrandbits(32) | 1 << 31 for _ in range(la)]
                bl = [rng.getrandbits(32) | 1 << 31 for _ in range(lb)]
            else:
                al, bl = [0xFFFFFFFF] * la, [0xFFFFFFFF] * lb
            kl = [rng.getrandbits(32) | 1 for _ in range(3)]
            a, b, k = _big(ck, al), _big(ck, bl), _big(ck, kl)
            want = R.biguint_mul(al, bl)
            assert a.mul(b, COMPAT).decrypt_limbs(ck) == want, (la, lb, trial)
            assert a.mul_add(b, k, COMPAT).decrypt_limbs(ck) == R.biguint_add(kl, want), (la, lb, trial)


def test_biguint_compat_chain_shapes_and_boundaries(keys):
    """The compat carry-count chain (csrc/compat_chain.cpp) on the GPU: shapes 2x8, 8x2 and 8x12 (the
    shorter side decides), limbs at the 2^32 boundaries the chain's near / g logic keys on (2^32 - 1,
    - 2, - 16, - 17, 15, 16) -- decrypted limbs equal to the reference's loop; 9x9 (outside the chain's
    range) goes through the dependency-wave form."""
    ck, _ = keys
    M = 1 << 32
    special = [M - 1, M - 2, M - 16, M - 17, 15, 16, 0]
    rng = random.Random(0xC4A1)
    cases = [(2, 8), (8, 2), (8, 12), (9, 9)]
    for la, lb in cases:
        al = [rng.choice(special + [rng.getrandbits(32)]) for _ in range(la)]
        bl = [rng.choice(special + [rng.getrandbits(32)]) for _ in range(lb)]
        al[-1] |= 1  # no leading zero limb (BigUintFHE::new drops them)
        bl[-1] |= 1
        want = R.biguint_mul(al, bl)
        a, b = _big(ck, al), _big(ck, bl)
        got = a.mul(b, COMPAT).decrypt_limbs(ck)
        assert got == want, (la, lb)


def test_random_op_chains(keys):
    """Seeded random chains of radix ops on the GPU (ciphertext outputs feeding later ops, widths 8 to
    128 bits, encrypted and clear operands), every intermediate decrypted against exact tfhe
    semantics: wrapping + - *, & (encrypted and clear), encrypted >> <<, min / max / <, / and % by clear
    and encrypted divisors (x / 0 = all ones, x % 0 = x)."""
    from fhe_sign import FheUint
    ck, _ = keys
    rng = random.Random(0xC4A1)
    for bits in (8, 16, 32, 64, 128):
        M = (1 << bits) - 1
        vals = [rng.getrandbits(bits) for _ in range(3)] + [0, M]
        enc = [FheUint.try_encrypt(v, ck, bits=bits) for v in vals]
        for step in range(25):
            i, j = rng.randrange(len(vals)), rng.randrange(len(vals))
            x, y, X, Y = vals[i], vals[j], enc[i], enc[j]
            op = rng.choice(["add", "sub", "mul", "and", "andc", "shr", "shl", "min", "max", "lt", "divc", "remc",
                             "div", "rem"] if bits <= 64 else ["add", "sub", "and", "shr", "min", "lt", "divc"])
            c = rng.getrandbits(max(2, bits // 2)) | 1
            s = y % bits
            want, got = {
                "add": (lambda: ((x + y) & M, X + Y)), "sub": (lambda: ((x - y) & M, X - Y)),
                "mul": (lambda: ((x * y) & M, X * Y)), "and": (lambda: (x & y, X & Y)),
                "andc": (lambda: (x & c, X & c)),
                "shr": (lambda: (x >> s, X >> Y)), "shl": (lambda: ((x << s) & M, X << Y)),
                "min": (lambda: (min(x, y), X.min(Y))), "max": (lambda: (max(x, y), X.max(Y))),
                "lt": (lambda: (int(x < y), X.lt(Y))), "divc": (lambda: (x // c, X / c)),
                "remc": (lambda: (x % c, X % c)),
                "div": (lambda: (x // y if y else M, X // Y)), "rem": (lambda: (x % y if y else x, X % Y)),
            }[op]()
            assert got.decrypt(ck) == want, (bits, step, op, hex(x), hex(y))
            if op not in ("lt",):  # feed the result into later steps
                vals.append(want)
                enc.append(got)
