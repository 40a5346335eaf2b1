"""Schnorr / BIP-340 signer (src/schnorr.rs) over the C ABI.

`Schnorr` mirrors the reference struct: sign, sign_with_k0, sign_fhe, sign_fhe_with_k0, verify,
plus compute_nonce / get_public_key_with_even_y.  Scalars are Python ints; signatures bytes.
"""
from __future__ import annotations

import ctypes as C

from ._lib import check, load
from .integer import COMPAT, _ctx


CURVE_ORDER = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141  # secp256k1 n


def _b32(x: int) -> bytes:
    return int(x).to_bytes(32, "big")


def _buf(b: bytes):
    return (C.c_uint8 * max(len(b), 1)).from_buffer_copy(b if b else b"\0")


def public_key_x(privkey: int) -> bytes:
    out = (C.c_uint8 * 32)()
    check(load().fhe_schnorr_public_key(_buf(_b32(privkey)), out))
    return bytes(out)


def compute_nonce(privkey: int, message: bytes, aux_rand: bytes) -> int:
    out = (C.c_uint8 * 32)()
    check(load().fhe_schnorr_compute_nonce(_buf(_b32(privkey)), _buf(message), len(message), _buf(aux_rand), out))
    return int.from_bytes(bytes(out), "big")


class Schnorr:
    def sign(self, message: bytes, aux_rand: bytes, privkey: int) -> bytes:
        sig = (C.c_uint8 * 64)()
        check(load().fhe_schnorr_sign(_buf(message), len(message), _buf(aux_rand), _buf(_b32(privkey)), sig))
        return bytes(sig)

    def sign_with_k0(self, message: bytes, k0: int, privkey: int) -> bytes:
        sig = (C.c_uint8 * 64)()
        check(load().fhe_schnorr_sign_with_k0(_buf(message), len(message), _buf(_b32(k0)), _buf(_b32(privkey)), sig))
        return bytes(sig)

    def sign_prologue(self, message: bytes, k0: int, privkey: int):
        """(k, e, r_x) of sign_fhe_with_k0's plaintext steps 1-5 (src/schnorr.rs:239-267)"""
        k, e, rx = (C.c_uint8 * 32)(), (C.c_uint8 * 32)(), (C.c_uint8 * 32)()
        check(load().fhe_schnorr_sign_prologue(_buf(message), len(message), _buf(_b32(k0)), _buf(_b32(privkey)), k, e,
                                               rx))
        return int.from_bytes(bytes(k), "big"), int.from_bytes(bytes(e), "big"), bytes(rx)

    def sign_fhe_with_k0_callsite(self, message: bytes, k0: int, privkey: int, privkey_fhe, client_key,
                                  mode: int = COMPAT) -> bytes:
        """sign_fhe_with_k0 exactly as the reference's call site runs it (src/schnorr.rs:271-276), each
        operator through its own C entry point -- what INTEGRATION.md 2's impl Add / impl Mul binding
        dispatches: e_fhe = BigUintFHE::new(e), k_fhe = BigUintFHE::new(k), k_fhe + (e_fhe * privkey_fhe),
        to_biguint, % n.  Signature identical to sign_fhe_with_k0 (which fuses the block into one
        column-form schedule)."""
        from .integer import BigUintFHE
        k, e, rx = self.sign_prologue(message, k0, privkey)
        e_fhe = BigUintFHE.new(e, client_key)
        k_fhe = BigUintFHE.new(k, client_key)
        s_without_mod = k_fhe.add(e_fhe.mul(privkey_fhe, mode), mode).to_biguint(client_key)
        return rx + _b32(s_without_mod % CURVE_ORDER)

    def sign_fhe_with_k0(self, message: bytes, k0: int, privkey: int, privkey_fhe, client_key, mode: int = COMPAT) -> bytes:
        sig = (C.c_uint8 * 64)()
        check(load().fhe_schnorr_sign_fhe_with_k0(_ctx().handle, client_key.handle, _buf(message), len(message),
                                                  _buf(_b32(k0)), _buf(_b32(privkey)), privkey_fhe.handle, mode, sig))
        return bytes(sig)

    def sign_fhe_with_k0_batch(self, jobs, client_key, mode: int = COMPAT) -> list:
        """jobs: [(message, k0, privkey, privkey_fhe)]; one engine schedule for all, signatures
        identical to sign_fhe_with_k0 one by one"""
        n = len(jobs)
        bufs = [C.create_string_buffer(bytes(m), max(1, len(m))) for m, _, _, _ in jobs]
        msgs = (C.c_void_p * max(1, n))(*[C.cast(b, C.c_void_p) for b in bufs])
        lens = (C.c_size_t * max(1, n))(*[len(m) for m, _, _, _ in jobs])
        k0s = b"".join(_b32(k) for _, k, _, _ in jobs)
        pks = b"".join(_b32(d) for _, _, d, _ in jobs)
        fh = (C.c_void_p * max(1, n))(*[f.handle for _, _, _, f in jobs])
        sigs = C.create_string_buffer(64 * max(1, n))
        check(load().fhe_schnorr_sign_fhe_with_k0_batch(_ctx().handle, client_key.handle, n, msgs, lens, k0s, pks, fh,
                                                        mode, sigs))
        return [sigs.raw[64 * i:64 * i + 64] for i in range(n)]

    def sign_fhe(self, message: bytes, aux_rand: bytes, privkey: int, client_key, mode: int = COMPAT) -> bytes:
        sig = (C.c_uint8 * 64)()
        check(load().fhe_schnorr_sign_fhe(_ctx().handle, client_key.handle, _buf(message), len(message),
                                          _buf(aux_rand), _buf(_b32(privkey)), mode, sig))
        return bytes(sig)

    @staticmethod
    def verify(message: bytes, pubkey: bytes, sig: bytes) -> bool:
        return load().fhe_schnorr_verify(_buf(message), len(message), _buf(pubkey), len(pubkey), _buf(sig), len(sig)) == 1
