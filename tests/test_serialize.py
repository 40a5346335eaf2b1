"""Key and ciphertext serialization: this engine's own versioned, checksummed
format (include/fhe_rocm.h, csrc/serial.h).  The reference never serializes (src/schnorr.rs:47 is the
only `serial` hit, a doc comment) and tfhe-rs's bincode/versionable layout is parity-unpinned here (no
tfhe-rs fixture), so the bar is: exact round trips, continued encryption streams, and loud rejection
of corrupted, truncated, mislabelled or out-of-budget input.  CPU tests cover the keys; the GPU
tests cover device-resident ciphertexts (radix integers, BigUintFHE limb vectors)."""
import numpy as np
import pytest

from fhe_sign import (BigUintFHE, ClientKey, Context, FheUint32, FheUint256, ServerKey, generate_keys,
                      set_server_key)
from fhe_sign._lib import FheError

SEED = 0x5E71A1


@pytest.fixture(scope="module")
def keys():
    return generate_keys(seed=SEED)


def test_client_key_round_trip_and_stream(keys):
    ck, _ = keys
    ck.seed_encryption(5, 100)
    ck.encrypt_block(1)                      # advance the stream mid-block
    blob = ck.serialize()
    ck2 = ClientKey.deserialize(blob)
    for a, b in zip(ck.export(), ck2.export()):
        assert np.array_equal(a, b)
    assert ck2.params.lwe_dimension == ck.params.lwe_dimension
    # both continue the same encryption stream
    for m in (0, 3, 15):
        assert np.array_equal(ck.encrypt_block(m), ck2.encrypt_block(m))
    assert ck2.decrypt_block(ck2.encrypt_block(9)) == 9
    assert ClientKey.deserialize(ck2.serialize()).serialize() == ck2.serialize()


def test_server_key_round_trip(keys):
    _, sk = keys
    blob = sk.serialize()
    assert len(blob) > 100_000_000  # KSK + BSK, standard domain
    sk2 = ServerKey.deserialize(blob)
    for a, b in zip(sk.export(), sk2.export()):
        assert np.array_equal(a, b)


def _flip(blob, i):
    b = bytearray(blob)
    b[i] ^= 0x01
    return bytes(b)


def test_rejects_corrupt_truncated_and_mislabelled(keys):
    ck, _ = keys
    blob = ck.serialize()
    for bad in (_flip(blob, 0), _flip(blob, 9), _flip(blob, len(blob) // 2), blob[:-1], blob + b"\0",
                blob[:20], b""):
        with pytest.raises(FheError):
            ClientKey.deserialize(bad)
    with pytest.raises(FheError, match="kind"):
        ServerKey.deserialize(blob)


def test_rejects_non_binary_secret(keys):
    """a well-formed frame (valid checksum) whose secret key is not binary is still refused"""
    import struct
    from fhe_sign.core import load  # noqa: F401  (library loaded by the fixture)
    ck, _ = keys
    blob = bytearray(ck.serialize())
    off = 32 + 8 * 4 + 4                    # header, params, lwe length
    blob[off] = 2                           # lwe_sk[0] = 2
    payload = bytes(blob[32:])
    payload += b"\0" * (-len(payload) % 8)
    h = 0xcbf29ce484222325
    for (x,) in struct.iter_unpack("<Q", payload):
        h = ((h ^ x) * 0x100000001b3) & (2**64 - 1)
    blob[24:32] = struct.pack("<Q", h)
    with pytest.raises(FheError, match="malformed"):
        ClientKey.deserialize(bytes(blob))


@pytest.mark.gpu
def test_ciphertext_round_trip_gpu(keys):
    ck, sk = keys
    ctx = Context(0)
    ctx.set_server_key(ServerKey.deserialize(sk.serialize()))  # a server key loaded from bytes
    set_server_key(ctx)
    try:
        a, b = 0xF11E51 << 200 | 12345, 2**255 + 977
        A = FheUint256.try_encrypt(a, ck)
        A2 = FheUint256.deserialize(A.serialize())
        assert A2.bits == 256 and A2.decrypt(ck) == a
        assert (A2 + FheUint256.try_encrypt(b, ck)).decrypt(ck) == (a + b) % 2**256   # usable in ops
        T = FheUint32.try_encrypt(7, ck) & 0xFF00                                      # trivial blocks
        assert FheUint32.deserialize(T.serialize()).decrypt(ck) == 0
        X = BigUintFHE.new(a, ck)
        X2 = BigUintFHE.deserialize(X.serialize())
        assert X2.to_biguint(ck) == a
        with pytest.raises(FheError):
            FheUint256.deserialize(_flip(A.serialize(), 100))
        with pytest.raises(FheError, match="kind"):
            BigUintFHE.deserialize(A.serialize())
    finally:
        set_server_key(None)
        ctx.close()
