"""Schnorr / BIP-340 host code of the engine (fhe-sign_amd/csrc/schnorr.cpp) vs the reference
data: tests/golden/bip340_vectors.csv (= reference tests/test_vectors.csv) and the plaintext
restatement.  Plaintext paths need no GPU; sign_fhe* are in test_sign_gpu.py."""
import csv
import os

import pytest

import ref_semantics as R
from conftest import ROOT
from fhe_sign import Schnorr, compute_nonce, public_key_x

ROWS = list(csv.DictReader(open(os.path.join(ROOT, "tests", "golden", "bip340_vectors.csv"))))


@pytest.mark.parametrize("row", ROWS, ids=lambda r: r["index"])
def test_verify_csv(row):
    """test_schnorr_vectors (src/schnorr.rs:531), verification half."""
    ok = Schnorr.verify(bytes.fromhex(row["message"]), bytes.fromhex(row["public key"]), bytes.fromhex(row["signature"]))
    assert ok == (row["verification result"] == "TRUE")


@pytest.mark.parametrize("row", [r for r in ROWS if r["secret key"]], ids=lambda r: r["index"])
def test_sign_and_nonce(row):
    d = int(row["secret key"], 16)
    msg, aux = bytes.fromhex(row["message"]), bytes.fromhex(row["aux_rand"])
    s = Schnorr()
    sig = s.sign(msg, aux, d)
    assert sig == R.sign(msg, aux, d)  # same algorithm as the restatement, incl. F8
    if row["index"] != "3":
        assert sig.hex().upper() == row["signature"].upper()
        assert public_key_x(d).hex().upper() == row["public key"].upper()
    k0 = compute_nonce(d, msg, aux)
    assert k0 == R.compute_nonce(d % R.N, R.pubkey_even_y(d % R.N), msg, aux)
    # test_schnorr_with_k0 (src/schnorr.rs:514): sign == sign_with_k0(compute_nonce)
    assert s.sign_with_k0(msg, k0, d) == sig


def test_vector0_expected_signature():
    """test_schnorr_bip340 (src/schnorr.rs:495)."""
    sig = Schnorr().sign(bytes(32), bytes(32), 3)
    assert sig.hex().upper() == ("E907831F80848D1069A5371B402410364BDF1C5F8307B0084C55F1CE2DCA8215"
                                 "25F66A4A85EA8B71E482A74F382D2CE5EBEEE8FDB2172F477DF4900D310536C0")
    assert Schnorr.verify(bytes(32), public_key_x(3), sig)


@pytest.mark.parametrize("row", [r for r in ROWS if r["secret key"]], ids=lambda r: r["index"])
def test_sign_prologue(row):
    """fhe_schnorr_sign_prologue = sign_fhe_with_k0's plaintext steps 1-5 (src/schnorr.rs:239-267): the k,
    e and r_x that the reference's call site feeds to BigUintFHE::new, vs the restatement"""
    d = int(row["secret key"], 16) % R.N
    msg, aux = bytes.fromhex(row["message"]), bytes.fromhex(row["aux_rand"])
    k0 = compute_nonce(d, msg, aux)
    k, e, rx = Schnorr().sign_prologue(msg, k0, d)
    flow = R.sign_fhe_limb_flow(msg, k0, d)
    assert (R.to_u32_digits(k), R.to_u32_digits(e)) == (flow["k"], flow["e"])
    assert rx == R.b32(flow["r_x"]) == Schnorr().sign_with_k0(msg, k0, d)[:32]
    # the call site's arithmetic on these values gives the signature
    assert rx + R.b32((k + e * d) % R.N) == Schnorr().sign_with_k0(msg, k0, d)
