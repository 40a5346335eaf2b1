"""config 4: Schnorr::sign_fhe_with_k0 on the GPU engine == sign_with_k0 byte-for-byte
(test_schnorr_fhe_with_k0, src/schnorr.rs:469-492) and == the CSV signature (test_schnorr_fhe,
src/schnorr.rs:440-466)."""
import csv
import os

import pytest

from conftest import ROOT
from fhe_sign import (COMPAT, FAST, PUBLIC, BigUintFHE, Context, Schnorr, compute_nonce, generate_keys, multi_bit_params,
                      public_key_x, set_server_key)

pytestmark = pytest.mark.gpu
ROWS = {r["index"]: r for r in csv.DictReader(open(os.path.join(ROOT, "tests", "golden", "bip340_vectors.csv")))}


@pytest.fixture(scope="module", params=["classic", "multibit"])
def env(request):
    """classic (grouping 1) and multi-bit (grouping 2) blind rotation: identical signatures"""
    ck, sk = generate_keys(multi_bit_params() if request.param == "multibit" else None, seed=0x5167)
    ctx = Context(0)
    ctx.set_server_key(sk)
    set_server_key(ctx)
    yield ck
    set_server_key(None)
    ctx.close()


def _sign_case(ck, idx, mode):
    row = ROWS[idx]
    d = int(row["secret key"], 16)
    msg, aux = bytes.fromhex(row["message"]), bytes.fromhex(row["aux_rand"])
    k0 = compute_nonce(d, msg, aux)
    s = Schnorr()
    d_fhe = BigUintFHE.new(d, ck)
    sig_fhe = s.sign_fhe_with_k0(msg, k0, d, d_fhe, ck, mode)
    assert sig_fhe == s.sign_with_k0(msg, k0, d)
    assert Schnorr.verify(msg, public_key_x(d), sig_fhe)
    return sig_fhe, row


def test_sign_fhe_with_k0_vector0(env):
    sig, row = _sign_case(env, "0", COMPAT)
    assert sig.hex().upper() == row["signature"].upper()


def test_sign_fhe_with_k0_vector1_8x8_limbs(env):
    sig, row = _sign_case(env, "1", COMPAT)
    assert sig.hex().upper() == row["signature"].upper()


def test_sign_fhe_fast_mode_vector15(env):
    sig, row = _sign_case(env, "15", FAST)
    assert sig.hex().upper() == row["signature"].upper()


def test_sign_fhe_vector0(env):
    """sign_fhe (src/schnorr.rs:154): encrypts the private key itself."""
    sig = Schnorr().sign_fhe(bytes(32), bytes(32), 3, env)
    assert sig.hex().upper() == ROWS["0"]["signature"].upper()


@pytest.mark.parametrize("idx", ["0", "1", "2", "16", "17", "18"])
def test_sign_public_operands_mode(env, idx):
    """e and k kept clear; the signature must not change (CSV rows with a signature)."""
    sig, row = _sign_case(env, idx, PUBLIC)
    assert sig.hex().upper() == row["signature"].upper()


def test_biguint_to_radix(env):
    v = (1 << 255) | 0x1234_5678_9ABC
    x = BigUintFHE.new(v, env)
    assert x.to_radix(300).decrypt(env) == v
    assert x.to_radix(64).decrypt(env) == v & (2**64 - 1)


@pytest.mark.parametrize("mode", [COMPAT, PUBLIC])
def test_sign_fhe_with_k0_batch(env, mode):
    """config 5b on one GPU: several independent signatures as ONE engine schedule
    (fhe_schnorr_sign_fhe_with_k0_batch) -- each byte-identical to sign_with_k0 (and to the CSV
    where the reference's F8 deviation does not apply); 1-limb and 8-limb private keys mixed."""
    ck = env
    s = Schnorr()
    jobs, want = [], []
    for idx in ("0", "1", "2", "15", "3"):
        row = ROWS[idx]
        d = int(row["secret key"], 16)
        msg, aux = bytes.fromhex(row["message"]), bytes.fromhex(row["aux_rand"])
        k0 = compute_nonce(d, msg, aux)
        jobs.append((msg, k0, d, BigUintFHE.new(d, ck)))
        want.append(s.sign_with_k0(msg, k0, d))
    got = s.sign_fhe_with_k0_batch(jobs, ck, mode)
    assert got == want
    for idx, sig in zip(("0", "1", "2", "15"), got):
        assert sig.hex().upper() == ROWS[idx]["signature"].upper()


@pytest.mark.parametrize("idx", ["0", "1"])
def test_sign_fhe_with_k0_reference_call_site(env, idx):
    """the reference's unchanged call site (src/schnorr.rs:271-276: BigUintFHE::new(e), ::new(k),
    k_fhe + (e_fhe * privkey_fhe), to_biguint, % n) bound operator by operator to the C ABI
     == the fused signer == the CSV"""
    row = ROWS[idx]
    d = int(row["secret key"], 16)
    msg, aux = bytes.fromhex(row["message"]), bytes.fromhex(row["aux_rand"])
    k0 = compute_nonce(d, msg, aux)
    s = Schnorr()
    d_fhe = BigUintFHE.new(d, env)
    sig = s.sign_fhe_with_k0_callsite(msg, k0, d, d_fhe, env, COMPAT)
    assert sig.hex().upper() == row["signature"].upper()
    assert sig == s.sign_fhe_with_k0(msg, k0, d, d_fhe, env, COMPAT)
