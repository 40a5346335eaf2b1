"""GPU PBS pipeline (KS -> MS -> BR -> SE, fhe-sign_amd/csrc/pbs_kernels.hip) against the C
oracle (oracle/tfhe_oracle.c): bit-exact ciphertexts on identical keys and inputs, and
decryptions equal to f(m).  This is the bootstrap under every FheUint op of the reference
(src/biguint.rs:138,223,236,243,248; src/perf_test.rs:28-54).
"""
import numpy as np
import pytest

import oracle
from fhe_sign import Context, default_params, generate_keys, multi_bit_params

pytestmark = pytest.mark.gpu
SEED = 0xC0FFEE


@pytest.fixture(scope="module", params=["classic", "multibit"])
def env(request):
    """every test runs on both blind rotations: classic (grouping 1, one CMUX per key bit) and
    multi-bit (grouping 2: oracle fho_blind_rotate's key-bundle path)"""
    mb = request.param == "multibit"
    ck, sk = generate_keys(multi_bit_params() if mb else None, seed=SEED)
    ok = oracle.OracleKeys(SEED, oracle.multibit_params() if mb else None)
    ctx = Context(0)
    ctx.set_server_key(sk)
    yield ck, sk, ok, ctx
    ctx.close()


def test_fourier_bsk_bit_exact(env):
    _, _, ok, ctx = env
    gpu = ctx.export_fourier_bsk()
    ref = oracle.fourier_bsk_gpu_layout(ok.bsk_f, ok.ggsw_count)
    assert gpu.shape == ref.shape
    bad = np.flatnonzero(gpu.view(np.uint64) != ref.view(np.uint64))
    assert bad.size == 0, f"{bad.size} mismatching doubles, first at {bad[:5]}"


def _luts():
    return [
        list(range(16)),                         # identity
        [m % 4 for m in range(16)],              # message extract
        [m // 4 for m in range(16)],             # carry extract
        [(m * m + 3) % 16 for m in range(16)],   # arbitrary
        [(m >> 2) * (m & 3) % 16 for m in range(16)],  # bivariate-style product
    ]


def test_pbs_bit_exact_vs_oracle(env):
    ck, _, ok, ctx = env
    tables = _luts()
    ids = [ctx.lut(t) for t in tables]
    r = ok.rng(4242)
    cts, lut_of, msgs = [], [], []
    for i in range(40):
        m = i % 16
        cts.append(ok.encrypt(r, m))
        lut_of.append(i % len(tables))
        msgs.append(m)
    cts = np.stack(cts)
    gpu = ctx.pbs(cts, np.array([ids[k] for k in lut_of], np.uint32))
    luts = np.stack([ok.make_lut(t) for t in tables])
    ref = ok.pbs_batch(cts, luts, np.array(lut_of, np.uint32))
    for i in range(len(cts)):
        assert np.array_equal(gpu[i], ref[i]), f"ciphertext {i} differs ({np.count_nonzero(gpu[i] != ref[i])} words)"
        assert ok.decrypt(gpu[i]) == tables[lut_of[i]][msgs[i]]


def test_full_bench_batch_sampled_vs_oracle(env):
    """bench.py's workload at its full size (BASELINE configs[1]: one level of 32768 blocks, the
    256-bit mul's widest): 32768 distinct encryptions through 5 LUTs in one launch of the throughput
    kernel; a seeded sample of 48 outputs bit-exact against the oracle, every 37th decrypting to f(m)."""
    ck, _, ok, ctx = env
    tables = _luts()
    ids = np.array([ctx.lut(t) for t in tables], np.uint32)
    B = 32768
    r = ok.rng(777)
    cts = np.stack([ok.encrypt(r, i % 16) for i in range(B)])
    lut_of = np.arange(B) % len(tables)
    gpu = ctx.pbs(cts, ids[lut_of])
    for i in range(0, B, 37):
        assert ok.decrypt(gpu[i]) == tables[lut_of[i]][i % 16], f"block {i}"
    pick = np.sort(np.random.default_rng(5).choice(B, 48, replace=False))
    luts = np.stack([ok.make_lut(t) for t in tables])
    ref = ok.pbs_batch(np.ascontiguousarray(cts[pick]), luts, lut_of[pick].astype(np.uint32))
    for k, i in enumerate(pick):
        assert np.array_equal(gpu[i], ref[k]), f"ciphertext {i} differs"


def test_pbs_chained_and_large_batch(env):
    """Repeated bootstrapping keeps decrypting correctly (noise is refreshed), and a batch larger
    than the chip's workgroup capacity (4096 ciphertexts) is handled."""
    ck, _, ok, ctx = env
    inc = ctx.lut([(m + 1) % 16 for m in range(16)])
    ck.seed_encryption(11)
    B = 4096
    ms = np.arange(B) % 16
    cts = np.stack([ck.encrypt_block(int(m)) for m in ms[:64]])
    cts = np.concatenate([cts] * (B // 64))
    out = cts
    for step in range(3):
        out = ctx.pbs(out, inc)
    dec = np.array([ck.decrypt_block(out[i]) for i in range(0, B, 97)])
    assert np.array_equal(dec, (ms[::97] + 3) % 16)
    # identical inputs give identical outputs (deterministic kernel)
    assert np.array_equal(out[0], out[64])


def test_pbs_empty_batch(env):
    _, _, _, ctx = env
    out = ctx.pbs(np.zeros((0, 2049), np.uint64), 0)
    assert out.shape == (0, 2049)


def test_latency_and_throughput_kernels_bit_identical(env):
    """The latency kernel (br_wide.hip, 8 waves per ciphertext) and the throughput kernel (4 waves,
    br_qy.hip) implement the same arithmetic: identical output words, equal to the oracle.  37
    ciphertexts: a ragged batch with every LUT.  The retired kernels are refused loudly."""
    _, _, ok, ctx = env
    tables = _luts()
    ids = [ctx.lut(t) for t in tables]
    r = ok.rng(777)
    cts = np.stack([ok.encrypt(r, i % 16) for i in range(37)])
    lut_ids = np.array([ids[i % len(ids)] for i in range(37)], np.uint32)
    for retired in (0, 1, 2, 3):  # NARROW (r1), QUAD (r3), PAIR (r2), QX (r4)
        with pytest.raises(Exception, match="retired"):
            ctx.set_br_kernel(retired)
    try:
        ctx.set_wide_threshold(0)
        thr = ctx.pbs(cts, lut_ids)
        ctx.set_wide_threshold(1 << 30)
        wide = ctx.pbs(cts, lut_ids)
    finally:
        ctx.set_wide_threshold(256)
    assert np.array_equal(thr, wide)
    ref = ok.pbs_batch(cts[:6], np.stack([ok.make_lut(t) for t in tables]), np.arange(6, dtype=np.uint32) % len(tables))
    assert np.array_equal(wide[:6], ref)


def test_zero_and_sparse_masks_both_kernels(env):
    """Ciphertexts whose modulus-switched mask is 0 at every key bit (trivial encryptions: mask 0,
    body m delta -- every CMUX is an a = 0 step, the kernels run it with e - 1 = 0 while the oracle
    skips it, reducing on the same schedule) and at half of them (a random encryption with every
    other mask word of the big LWE zeroed): both blind-rotate kernels equal the oracle word for word,
    and the trivial ones decrypt to f(m)."""
    _, _, ok, ctx = env
    tables = _luts()
    ids = np.array([ctx.lut(t) for t in tables], np.uint32)
    luts = np.stack([ok.make_lut(t) for t in tables])
    delta = ok.delta()
    triv = np.zeros((16, 2049), np.uint64)
    triv[:, 2048] = (np.arange(16, dtype=np.uint64) * np.uint64(delta))
    r = ok.rng(4711)
    sparse = np.stack([ok.encrypt(r, m) for m in range(8)])
    sparse[:, 0:2048:2] = 0
    cts = np.ascontiguousarray(np.concatenate([triv, sparse]))
    lut_of = (np.arange(len(cts)) % len(tables)).astype(np.uint32)
    ref = ok.pbs_batch(cts, luts, lut_of)
    try:
        for thr in (0, 1 << 30):  # throughput kernel, latency kernel
            ctx.set_wide_threshold(thr)
            got = ctx.pbs(cts, ids[lut_of])
            bad = [i for i in range(len(cts)) if not np.array_equal(got[i], ref[i])]
            assert not bad, f"threshold {thr}: ciphertexts {bad} differ from the oracle"
    finally:
        ctx.set_wide_threshold(256)
    for m in range(16):
        assert ok.decrypt(ref[m]) == tables[lut_of[m]][m]


def test_throughput_kernel_ragged_batches(env):
    """The throughput kernel (br_qy.hip) at ragged batches (1, 2, 3, 37, 259) with every LUT gives
    the latency kernel's and the oracle's words; FHE_BR_QY is accepted, unknown kinds are refused."""
    _, _, ok, ctx = env
    tables = _luts()
    ids = [ctx.lut(t) for t in tables]
    r = ok.rng(991)
    cts = np.stack([ok.encrypt(r, (3 * i + 1) % 16) for i in range(259)])
    lut_ids = np.array([ids[i % len(ids)] for i in range(259)], np.uint32)
    try:
        ctx.set_wide_threshold(1 << 30)
        wide = ctx.pbs(cts, lut_ids)
        ctx.set_br_kernel(4)
        ctx.set_wide_threshold(0)
        thr = {c: ctx.pbs(cts[:c], lut_ids[:c]) for c in (1, 2, 3, 37, 259)}
    finally:
        ctx.set_wide_threshold(256)
        ctx.set_br_kernel(7)
    for c, out in thr.items():
        bad = [i for i in range(c) if not np.array_equal(out[i], wide[i])]
        assert not bad, f"batch {c}: ciphertexts {bad[:5]} differ from the latency kernel"
    ref = ok.pbs_batch(cts[:6], np.stack([ok.make_lut(t) for t in tables]), np.arange(6, dtype=np.uint32) % len(tables))
    assert np.array_equal(thr[37][:6], ref)
    for bad_kind in (8, -1):
        with pytest.raises(Exception):
            ctx.set_br_kernel(bad_kind)


def test_throughput_kernel_full_batch(env):
    """br_qy.hip and the latency kernel on the same 4096 distinct encryptions (16 rounds of 256 CUs):
    every output word identical, a seeded sample of 8 equal to the oracle."""
    _, _, ok, ctx = env
    tables = _luts()
    ids = np.array([ctx.lut(t) for t in tables], np.uint32)
    B = 4096
    r = ok.rng(31337)
    cts = np.stack([ok.encrypt(r, i % 16) for i in range(B)])
    lut_of = np.arange(B) % len(tables)
    qy = ctx.pbs(cts, ids[lut_of])
    try:
        ctx.set_wide_threshold(1 << 30)
        wide = ctx.pbs(cts, ids[lut_of])
    finally:
        ctx.set_wide_threshold(256)
    bad = np.flatnonzero((wide != qy).any(axis=1))
    assert bad.size == 0, f"{bad.size} ciphertexts differ between qy and the latency kernel, first {bad[:5]}"
    pick = np.array([0, 1, 513, 1024, 2047, 2048, 3333, 4095])
    ref = ok.pbs_batch(np.ascontiguousarray(cts[pick]), np.stack([ok.make_lut(t) for t in tables]),
                       lut_of[pick].astype(np.uint32))
    for k, i in enumerate(pick):
        assert np.array_equal(qy[i], ref[k]), f"ciphertext {i} differs from the oracle"


def test_keyswitch_kernels_identical(env):
    """The int8 matrix-core keyswitch (ks_mfma.hip: byte-plane contraction) and the 64-bit VALU
    keyswitch are both exact: the bootstraps they feed give identical words, equal to the oracle.
    Batches of 1, 16, 37 (ragged tiles), 130 and 4160 (the blocked path, ragged)."""
    _, _, ok, ctx = env
    tables = _luts()
    ids = [ctx.lut(t) for t in tables]
    r = ok.rng(4242)
    base = np.stack([ok.encrypt(r, i % 16) for i in range(130)])
    for count in (1, 16, 37, 130, 4160):  # 4160: the blocked MFMA path (4 tiles per wave), ragged end
        cts = np.ascontiguousarray(np.resize(base, (count, base.shape[1])))
        lut_ids = np.array([ids[i % len(ids)] for i in range(count)], np.uint32)
        try:
            ctx.set_ks_kernel(0)
            valu = ctx.pbs(cts, lut_ids)
            ctx.set_ks_kernel(1)
            mfma = ctx.pbs(cts, lut_ids)
        finally:
            ctx.set_ks_kernel(1)
        assert np.array_equal(valu, mfma), count
    ref = ok.pbs_batch(cts[:4], np.stack([ok.make_lut(t) for t in tables]), np.arange(4, dtype=np.uint32) % len(tables))
    assert np.array_equal(mfma[:4], ref)


@pytest.mark.parametrize("lwe_bound", [44, 45])
def test_noise_budget_lwe_bound(lwe_bound):
    """The decode margin at the radix layer's largest input (22 units, as below) with the small key's
    TUniform bound at 44 and at 45 (tfhe 0.10's recalled value): keyswitch + modulus
    switch by the oracle on the same keys, the phase error's sigma in the 4096-domain (half step 64)
    printed and bounded at 8 sigma, and every input bootstrapped to the right carry by the GPU."""
    P, OP = default_params(), oracle.default_params()
    P.lwe_noise_log2 = OP.lwe_noise_log2 = lwe_bound
    ck, sk = generate_keys(P, seed=SEED)
    ok = oracle.OracleKeys(SEED, OP)
    ctx = Context(0)
    try:
        ctx.set_server_key(sk)
        sigma, worst = _radix_limit_margin(ok, ctx, 1024)
    finally:
        ctx.close()
    print(f"\nlwe TUniform 2^{lwe_bound}: 22-unit input after KS + MS: sigma {sigma:.2f}, max |err| {worst} "
          f"of the half step 64 ({64 / sigma:.1f} sigma)")
    assert worst < 64 and sigma * 8 < 64


def _radix_limit_margin(ok, ctx, N):
    """(sigma, max |error|) of 4 s0 + 2 s1 + s2 + c built from N x 4 GPU bootstrap outputs, after the
    oracle's keyswitch and modulus switch, in the 4096-domain; the GPU bootstraps each to its carry"""
    ident = ctx.lut(list(range(16)))
    rs = np.random.default_rng(5)
    s = rs.integers(0, 3, size=(3, N))
    c = rs.integers(0, 2, size=N)
    r = ok.rng(77)
    fresh = np.stack([ok.encrypt(r, int(v)) for v in np.concatenate([s.ravel(), c])])
    unit = ctx.pbs(fresh, ident).astype(np.uint64)
    s0, s1, s2, cb = unit[:N], unit[N:2 * N], unit[2 * N:3 * N], unit[3 * N:]
    with np.errstate(over="ignore"):
        comb = (np.uint64(4) * s0 + np.uint64(2) * s1 + s2 + cb).astype(np.uint64)
    m = 4 * s[0] + 2 * s[1] + s[2] + c
    n = ok.params.n
    sk = ok.lwe_sk.astype(np.int64)
    small = ok.keyswitch_batch(comb)
    ms = (((small[:, : n + 1].astype(object) + (1 << 51)) >> 52) % 4096).astype(np.int64)
    phase = (ms[:, n] - (ms[:, :n] * sk).sum(axis=1)) % 4096
    errs = ((phase - 128 * m + 2048) % 4096 - 2048).astype(np.float64)
    carry = ctx.lut([1 if v >= 8 else 0 for v in range(16)])
    out = ctx.pbs(comb, carry)
    assert [ok.decrypt(o) for o in out] == [int(v >= 8) for v in m]
    return float(errs.std()), int(np.abs(errs).max())


def test_noise_budget_at_radix_limit(env):
    """The radix layer admits PBS inputs up to kMaxNoise = 25 fresh-bootstrap variances (sigma <= 5
    fresh sigmas, tfhe-rs' max noise level 5 for 2_2).  Its largest real input is the carry prefix's
    4 s0 + 2 s1 + s2 + c (22 units, csrc/radix.cpp:carry_prefix).  Built here from GPU bootstrap
    outputs, keyswitched and modulus-switched by the oracle: the phase error in the 4096-domain
    stays far inside the half step (64), and every such input bootstraps to the right value."""
    _, _, ok, ctx = env
    ident = ctx.lut(list(range(16)))
    rs = np.random.default_rng(5)
    N = 384
    s = rs.integers(0, 3, size=(3, N))
    c = rs.integers(0, 2, size=N)
    r = ok.rng(77)
    fresh = np.stack([ok.encrypt(r, int(v)) for v in np.concatenate([s.ravel(), c])])
    unit = ctx.pbs(fresh, ident).astype(np.uint64)  # unit-noise blocks (fresh bootstrap outputs)
    s0, s1, s2, cb = unit[:N], unit[N:2 * N], unit[2 * N:3 * N], unit[3 * N:]
    with np.errstate(over="ignore"):
        comb = (np.uint64(4) * s0 + np.uint64(2) * s1 + s2 + cb).astype(np.uint64)
    m = 4 * s[0] + 2 * s[1] + s[2] + c
    n = ok.params.n
    sk = ok.lwe_sk.astype(object)
    errs = []
    for i in range(N):
        small = ok.keyswitch(comb[i])
        ms = [((int(w) + (1 << 51)) >> 52) % 4096 for w in small[: n + 1]]
        phase = (ms[n] - sum(a * b for a, b in zip(ms[:n], sk))) % 4096
        errs.append((phase - 128 * int(m[i]) + 2048) % 4096 - 2048)
    errs = np.array(errs, dtype=np.float64)
    assert np.abs(errs).max() < 64
    assert errs.std() * 8 < 64, f"modulus-switched sigma {errs.std():.2f} leaves < 8 sigma of margin"
    carry = ctx.lut([1 if v >= 8 else 0 for v in range(16)])
    out = ctx.pbs(comb, carry)
    assert [ok.decrypt(o) for o in out] == [int(v >= 8) for v in m]


def test_multibit_qy_kernel_bit_identical():
    """br_qy.hip's multi-bit instance (the key bundle per point of phase E, built during the forward
    transform) gives the multi-bit latency kernel's and the oracle's words, at ragged batches and at
    4096 distinct encryptions (16 rounds of 256 CUs)."""
    mb = multi_bit_params()
    ck, sk = generate_keys(mb, seed=SEED)
    ok = oracle.OracleKeys(SEED, oracle.multibit_params())
    tables = _luts()
    r = ok.rng(2024)
    B = 4096
    cts = np.stack([ok.encrypt(r, (7 * i + 2) % 16) for i in range(B)])
    lut_of = np.arange(B) % len(tables)
    ctx = Context(0)
    try:
        ctx.set_server_key(sk)
        ids = np.array([ctx.lut(t) for t in tables], np.uint32)
        ctx.set_wide_threshold(1 << 30)
        wide = ctx.pbs(cts, ids[lut_of])
        ctx.set_wide_threshold(0)
        got = {c: ctx.pbs(cts[:c], ids[lut_of[:c]]) for c in (1, 37, 259)}
        full = ctx.pbs(cts, ids[lut_of])
    finally:
        ctx.close()
    for c, out in got.items():
        bad = np.flatnonzero((out != wide[:c]).any(axis=1))
        assert bad.size == 0, f"batch {c}: ciphertexts {bad[:5]} differ from the latency kernel"
    bad = np.flatnonzero((full != wide).any(axis=1))
    assert bad.size == 0, f"{bad.size} ciphertexts differ between qy<2> and the latency kernel, first {bad[:5]}"
    pick = np.array([0, 1, 777, 2048, 4095])
    ref = ok.pbs_batch(np.ascontiguousarray(cts[pick]), np.stack([ok.make_lut(t) for t in tables]),
                       lut_of[pick].astype(np.uint32))
    for k, i in enumerate(pick):
        assert np.array_equal(full[i], ref[k]), f"ciphertext {i} differs from the oracle"


def test_two_ciphertext_kernel_bit_identical():
    """k_blind_rotate_qy2 (FHE_BR_QY2: two ciphertexts per workgroup sharing each key slice; FHE_BR_QY4: two
    such pairs per 8-wave workgroup) gives qy's and the oracle's words at every batch residue (a pair
    with one ciphertext runs it twice and stores it once; a half with none still joins the barriers)."""
    ck, sk = generate_keys(seed=SEED)
    ok = oracle.OracleKeys(SEED)
    tables = _luts()
    r = ok.rng(99)
    B = 1031
    cts = np.stack([ok.encrypt(r, (5 * i + 3) % 16) for i in range(B)])
    lut_of = np.arange(B) % len(tables)
    ctx = Context(0)
    try:
        ctx.set_server_key(sk)
        ids = np.array([ctx.lut(t) for t in tables], np.uint32)
        ctx.set_wide_threshold(0)
        got = {}
        for kind in (4, 5, 6):
            ctx.set_br_kernel(kind)
            got[kind] = {c: ctx.pbs(cts[:c], ids[lut_of[:c]]) for c in (1, 2, 3, 5, 6, 258, B)}
        ctx.set_br_kernel(7)
    finally:
        ctx.close()
    for kind in (5, 6):
        for c in got[4]:
            bad = np.flatnonzero((got[4][c] != got[kind][c]).any(axis=1))
            assert bad.size == 0, f"kind {kind}, batch {c}: ciphertexts {bad[:5]} differ from qy"
    pick = np.array([0, 1, 2, 515, 1030])
    ref = ok.pbs_batch(np.ascontiguousarray(cts[pick]), np.stack([ok.make_lut(t) for t in tables]),
                       lut_of[pick].astype(np.uint32))
    for k, i in enumerate(pick):
        assert np.array_equal(got[5][B][i], ref[k]), f"ciphertext {i} differs from the oracle"
