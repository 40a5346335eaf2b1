"""Schnorr / BIP-340 signer (src/schnorr.rs) over the C ABI.

`Schnorr` mirrors the reference struct: sign, sign_with_k0, sign_fhe, sign_fhe_with_k0, verify,
plus compute_nonce / get_public_key_with_even_y.  Scalars are Python ints; signatures bytes.
"""
from __future__ import annotations

import ctypes as C

from ._lib import check, load
from .integer import COMPAT, _ctx


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
