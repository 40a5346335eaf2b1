"""Product keygen / encryption (fhe-sign_amd, C++) vs the oracle's restatement (C): byte-identical.

Reference call sites: tfhe::generate_keys (src/schnorr.rs:441-442), FheUint32::try_encrypt
(src/biguint.rs:26).  Key bytes against tfhe-rs itself: parity unpinned (no tfhe-rs fixture).
"""
import numpy as np
import pytest

import oracle
from fhe_sign import generate_keys

SEED = 0x5EED_F11E


@pytest.fixture(scope="module")
def keys():
    ck, sk = generate_keys(seed=SEED)
    ok = oracle.OracleKeys(SEED)
    return ck, sk, ok


def test_secret_keys_identical(keys):
    ck, _, ok = keys
    lwe, glwe = ck.export()
    assert np.array_equal(lwe, ok.lwe_sk)
    assert np.array_equal(glwe, ok.glwe_sk)
    assert set(np.unique(lwe)) <= {0, 1} and 300 < lwe.sum() < 534


def test_server_keys_identical(keys):
    _, sk, ok = keys
    ksk, bsk = sk.export()
    assert np.array_equal(ksk, ok.ksk)
    assert np.array_equal(bsk, ok.bsk)


def test_encryption_identical_and_decrypts(keys):
    ck, _, ok = keys
    ck.seed_encryption(77, 100)
    r = ok.rng(77, 100)
    for m in range(16):
        a = ck.encrypt_block(m)
        b = ok.encrypt(r, m)
        assert np.array_equal(a, b)
        assert ck.decrypt_block(a) == m
        assert ok.decrypt(b) == m


def test_ksk_rows_decrypt_to_gadget(keys):
    """KSK[j][l] is an LWE encryption of S_j * 2^(64 - 3(l+1)) under the small key."""
    _, _, ok = keys
    n, L = ok.params.n, ok.params.ks_level
    ksk = ok.ksk.reshape(2048, L, n + 1)
    for j in (0, 1, 777, 2047):
        for lv in range(L):
            row = ksk[j, lv]
            phase = (int(row[n]) - int(np.dot(row[:n].astype(object), ok.lwe_sk.astype(object)))) % 2**64
            expect = (int(ok.glwe_sk[j]) << (64 - 3 * (lv + 1))) % 2**64
            err = (phase - expect + 2**63) % 2**64 - 2**63
            assert abs(err) <= 2**ok.params.lwe_noise_log2


def test_batch_encryption_equals_sequential():
    """fhe_encrypt_blocks (multi-threaded over seeked copies of the encryption stream, used by every
    radix / BigUintFHE encryption) gives the sequential loop's ciphertexts and leaves the stream where
    the loop would, for batch sizes around the threading threshold and a stream mid-block."""
    import numpy as np
    from fhe_sign import generate_keys
    ck, _ = generate_keys(seed=0xB1)
    ck2, _ = generate_keys(seed=0xB1)
    for n in (1, 31, 64, 257, 1000):
        ck.seed_encryption(n, 100)
        ck2.seed_encryption(n, 100)
        ck.encrypt_block(3)  # start mid-way through a ChaCha block
        ck2.encrypt_block(3)
        vals = [(7 * i + n) % 16 for i in range(n)]
        seq = np.stack([ck.encrypt_block(v) for v in vals])
        bat = ck2.encrypt_blocks(vals)
        assert np.array_equal(seq, bat), n
        assert np.array_equal(ck.encrypt_block(5), ck2.encrypt_block(5))  # same stream position after
        assert [ck2.decrypt_block(c) for c in bat[:20]] == vals[:20]


def test_default_keys_are_drawn_from_os_entropy():
    """generate_keys() with no seed keys every stream with 32 bytes of os.urandom (tfhe-rs draws from
    the OS CSPRNG, src/schnorr.rs:441-442): two calls give unrelated secret keys, and the keyed C
    entry with the bytes of a test seed's public expansion {seed, "FHES", 0...} rebuilds exactly the
    seeded (deterministic, insecure) keys -- the seed path is only a fixed key, not a weaker cipher."""
    import ctypes as C
    import struct

    from fhe_sign._lib import check, load
    from fhe_sign.core import ClientKey, ServerKey, default_params

    a, _ = generate_keys()
    b, _ = generate_keys()
    la, ga = a.export()
    lb, gb = b.export()
    assert not np.array_equal(la, lb) and not np.array_equal(ga, gb)
    assert 300 < la.sum() < 534

    seed = 0xB1
    key = struct.pack("<8I", seed & 0xFFFFFFFF, seed >> 32, 0x46484553, 0, 0, 0, 0, 0)
    p = default_params()
    ck, sk = C.c_void_p(), C.c_void_p()
    check(load().fhe_generate_keys_keyed(C.byref(p), (C.c_uint8 * 32).from_buffer_copy(key), C.byref(ck),
                                         C.byref(sk)))
    ck, sk = ClientKey(ck, p), ServerKey(sk, p)
    ref_ck, ref_sk = generate_keys(seed=seed)
    for x, y in zip(ck.export(), ref_ck.export()):
        assert np.array_equal(x, y)
    for x, y in zip(sk.export(), ref_sk.export()):
        assert np.array_equal(x, y)
    assert load().fhe_generate_keys_keyed(C.byref(p), None, C.byref(ck.handle), C.byref(sk.handle)) != 0
