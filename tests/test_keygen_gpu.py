"""Server-key generation on the GPU (fhe_generate_keys_device, keygen.hip)
against the oracle's keygen restatement (oracle/tfhe_oracle.c, the same ChaCha20 streams): every
key word identical.  Reference call site: tfhe::generate_keys (src/schnorr.rs:441-442); key bytes
against tfhe-rs itself: parity unpinned (no tfhe-rs fixture)."""
import time

import numpy as np
import pytest

import oracle
from fhe_sign import Context, generate_keys, multi_bit_params

pytestmark = pytest.mark.gpu

SEED = 0x5EED_F11E


@pytest.fixture(scope="module")
def ctx():
    return Context(0)


def test_device_keys_equal_oracle(ctx):
    t = time.perf_counter()
    ck, sk = generate_keys(seed=SEED, device=ctx)
    dt = time.perf_counter() - t
    ok = oracle.OracleKeys(SEED)
    lwe, glwe = ck.export()
    assert np.array_equal(lwe, ok.lwe_sk) and np.array_equal(glwe, ok.glwe_sk)
    ksk, bsk = sk.export()
    assert np.array_equal(ksk, ok.ksk)
    assert np.array_equal(bsk, ok.bsk)
    print(f"device keygen {dt * 1e3:.1f} ms (incl. download)")


@pytest.mark.parametrize("seed", [0, 2**64 - 1])
def test_device_keys_equal_host(ctx, seed):
    _, sk_h = generate_keys(seed=seed)
    _, sk_d = generate_keys(seed=seed, device=ctx)
    kh, bh = sk_h.export()
    kd, bd = sk_d.export()
    assert np.array_equal(kh, kd) and np.array_equal(bh, bd)


def test_device_key_bootstraps(ctx):
    ck, sk = generate_keys(seed=9, device=ctx)
    ctx.set_server_key(sk)
    lid = ctx.lut([(3 * m + 1) % 16 for m in range(16)])
    cts = np.stack([ck.encrypt_block(m) for m in range(16)])
    out = ctx.pbs(cts, lid)
    assert [ck.decrypt_block(o) for o in out] == [(3 * m + 1) % 16 for m in range(16)]


def test_device_multibit_keys_equal_oracle(ctx):
    """multi-bit bootstrapping key (grouping 2: GGSWs of the pattern indicators f_B of each pair of
    key bits) generated on the GPU == the oracle's, word for word; and a fresh random (os.urandom)
    key generated on the device equals the host keygen of the same 256-bit key"""
    ck, sk = generate_keys(multi_bit_params(), seed=SEED, device=ctx)
    ok = oracle.OracleKeys(SEED, oracle.multibit_params())
    ksk, bsk = sk.export()
    assert bsk.size == ok.bsk.size == 417 * 3 * 4 * 2048
    assert np.array_equal(ksk, ok.ksk) and np.array_equal(bsk, ok.bsk)
    ctx.set_server_key(sk)
    lid = ctx.lut([(5 * m + 2) % 16 for m in range(16)])
    cts = np.stack([ck.encrypt_block(m) for m in range(16)])
    out = ctx.pbs(cts, lid)
    assert [ck.decrypt_block(o) for o in out] == [(5 * m + 2) % 16 for m in range(16)]
