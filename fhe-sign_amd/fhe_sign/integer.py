"""FheUint{8,32,64} and BigUintFHE: the reference's encrypted-integer surface over the C ABI.

Mirrors the operator set coset-io/fhe-sign uses on tfhe's high-level types
(src/biguint.rs:108-117,135-143,221-248; src/perf_test.rs:19-56) and the BigUintFHE struct
(src/biguint.rs:8-265).  Operators do not consume their inputs (Rust consumed them; callers
cloned, src/schnorr.rs:274).  The server side is an explicit Context (tfhe's thread-local
set_server_key, src/schnorr.rs:443, is `set_server_key(ctx)` here).
"""
from __future__ import annotations

import ctypes as C
import threading

import numpy as np

from ._lib import check, load, ptr, serialize_with

COMPAT = 0  # exact replay of src/biguint.rs:214-254 incl. the wrapping add at :247-249
FAST = 1    # true product/sum, single wide carry propagation
PUBLIC = 2  # signer only: e and k stay clear, s = e * Enc(d') + k as a wide scalar multiply-add

_tls = threading.local()


def set_server_key(ctx) -> None:
    """tfhe::set_server_key (src/schnorr.rs:443): the context used by operators on this thread."""
    _tls.ctx = ctx


def _ctx():
    ctx = getattr(_tls, "ctx", None)
    if ctx is None:
        raise RuntimeError("no server key set on this thread (call set_server_key(ctx))")
    return ctx


def _hval(h):
    """the address of a handle (c_void_p or int)"""
    return h.value if isinstance(h, C.c_void_p) else h


def _words(value: int, bits: int) -> np.ndarray:
    n = (bits + 63) // 64
    v = value % (1 << bits)
    return np.array([(v >> (64 * i)) & (2**64 - 1) for i in range(n)], dtype=np.uint64)


class FheUint:
    BITS = 0

    def __init__(self, handle, bits=None):
        self._h = handle
        self.bits = bits or self.BITS

    @property
    def handle(self):
        return self._h

    def __del__(self):
        if getattr(self, "_h", None):
            load().fhe_radix_destroy(self._h)
            self._h = None

    @classmethod
    def _wrap(cls, h, bits):
        kind = {8: FheUint8, 32: FheUint32, 64: FheUint64, 128: FheUint128, 256: FheUint256, 2: FheBool}.get(bits, FheUint)
        obj = kind.__new__(kind)
        FheUint.__init__(obj, h, bits)
        return obj

    @classmethod
    def try_encrypt(cls, value: int, client_key, bits=None):
        bits = bits or cls.BITS
        ctx = _ctx()
        w = _words(value, bits)
        h = C.c_void_p()
        check(load().fhe_radix_encrypt(ctx.handle, client_key.handle, ptr(w), bits, C.byref(h)))
        return cls._wrap(h, bits)

    encrypt = try_encrypt

    @classmethod
    def encrypt_trivial(cls, value: int, bits=None):
        bits = bits or cls.BITS
        w = _words(value, bits)
        h = C.c_void_p()
        check(load().fhe_radix_trivial(_ctx().handle, ptr(w), bits, C.byref(h)))
        return cls._wrap(h, bits)

    def decrypt(self, client_key) -> int:
        n = (self.bits + 63) // 64
        w = np.zeros(n, np.uint64)
        check(load().fhe_radix_decrypt(_ctx().handle, client_key.handle, self._h, ptr(w), n))
        return sum(int(w[i]) << (64 * i) for i in range(n))

    def clone(self):
        h = C.c_void_p()
        check(load().fhe_radix_clone(self._h, C.byref(h)))
        return self._wrap(h, self.bits)

    @classmethod
    def broadcast(cls, x, root: int = 0, ctx=None):
        """Collective (fhe_ctx_broadcast_radix): rank `root` passes its FheUint, every other rank
        passes None and receives a copy with byte-identical block ciphertexts (RCCL over xGMI)."""
        ctx = ctx or _ctx()
        h = C.c_void_p(_hval(x.handle) if x is not None else None)
        check(load().fhe_ctx_broadcast_radix(ctx.handle, C.byref(h), root))
        if x is not None and h.value == _hval(x.handle):
            return x
        bits = C.c_uint32()
        check(load().fhe_radix_num_bits(h, C.byref(bits)))
        return cls._wrap(h, int(bits.value))

    def export(self) -> np.ndarray:
        nb = self.bits // 2
        out = np.zeros(nb * 2049, np.uint64)
        check(load().fhe_radix_export(_ctx().handle, self._h, ptr(out), out.size))
        return out.reshape(nb, 2049)

    # ---- helpers
    def _bin(self, fn, other):
        h = C.c_void_p()
        check(getattr(load(), fn)(_ctx().handle, self._h, other._h, C.byref(h)))
        return self._wrap(h, self.bits)

    def _scalar(self, fn, s):
        h = C.c_void_p()
        check(getattr(load(), fn)(_ctx().handle, self._h, s, C.byref(h)))
        return self._wrap(h, self.bits)

    def _scalar_any(self, fn, s: int, wrap: bool = True):
        """u64 entry point when the clear operand fits, the _words one otherwise (wide FheUint)."""
        s = int(s)
        if wrap:
            s %= 1 << self.bits
        if s < 0:
            raise ValueError("clear operand must be non-negative")
        if s < 2**64:
            return self._scalar(fn, s)
        w = _words(s, max(64, s.bit_length()))
        h = C.c_void_p()
        check(getattr(load(), fn + "_words")(_ctx().handle, self._h, ptr(w), w.size, C.byref(h)))
        return self._wrap(h, self.bits)

    # ---- operators (tfhe HL API)
    def __add__(self, o):
        return self._bin("fhe_radix_add", o) if isinstance(o, FheUint) else self._scalar_any("fhe_radix_scalar_add", o)

    def __sub__(self, o):
        return self._bin("fhe_radix_sub", o)

    def __mul__(self, o):
        return self._bin("fhe_radix_mul", o) if isinstance(o, FheUint) else self._scalar_any("fhe_radix_scalar_mul", o)

    def scalar_mul_add(self, m: int, k: int):
        """self * m + k for clear m, k (wrapping), one carry propagation"""
        wm, wk = _words(m, self.bits), _words(k, self.bits)
        h = C.c_void_p()
        P = C.POINTER(C.c_uint64)
        check(load().fhe_radix_scalar_mul_add_words(_ctx().handle, self._h, wm.ctypes.data_as(P), len(wm),
                                                     wk.ctypes.data_as(P), len(wk), C.byref(h)))
        return self._wrap(h, self.bits)

    def __and__(self, o):
        return self._bin("fhe_radix_bitand", o) if isinstance(o, FheUint) else self._scalar_any("fhe_radix_scalar_and", o)

    def __rshift__(self, o):
        if isinstance(o, FheUint):
            return self._bin("fhe_radix_shr", o)
        return self._scalar("fhe_radix_scalar_shr", int(o) % 2**32)

    def __lshift__(self, o):
        if isinstance(o, FheUint):
            return self._bin("fhe_radix_shl", o)
        return self._scalar("fhe_radix_scalar_shl", int(o) % 2**32)

    def __floordiv__(self, d):
        if isinstance(d, FheUint):
            return self._bin("fhe_radix_div", d)
        return self._scalar_any("fhe_radix_scalar_div", d, wrap=False)

    __truediv__ = __floordiv__  # tfhe's `&a / 5` on FheUint is integer division (src/perf_test.rs:54)

    def __mod__(self, d):
        if isinstance(d, FheUint):
            return self._bin("fhe_radix_rem", d)
        return self._scalar_any("fhe_radix_scalar_rem", d, wrap=False)

    def serialize(self) -> bytes:
        """ciphertext bytes (own format, include/fhe_rocm.h); restore with FheUint.deserialize"""
        return serialize_with(load().fhe_radix_serialize, _ctx().handle, self._h)

    @classmethod
    def deserialize(cls, data: bytes):
        h = C.c_void_p()
        check(load().fhe_radix_deserialize(_ctx().handle, data, len(data), C.byref(h)))
        bits = C.c_uint32(0)
        check(load().fhe_radix_num_bits(h, C.byref(bits)))
        return FheUint._wrap(h, bits.value)

    def div_rem(self, d):
        """(self // d, self % d) for an encrypted divisor, one pass"""
        q, r = C.c_void_p(), C.c_void_p()
        check(load().fhe_radix_divrem(_ctx().handle, self._h, d._h, C.byref(q), C.byref(r)))
        return self._wrap(q, self.bits), self._wrap(r, self.bits)

    def min(self, o):
        return self._bin("fhe_radix_min", o)

    def max(self, o):
        return self._bin("fhe_radix_max", o)

    def lt(self, o):
        h = C.c_void_p()
        check(load().fhe_radix_lt(_ctx().handle, self._h, o._h, C.byref(h)))
        return self._wrap(h, 2)

    def cast_into(self, cls):
        bits = cls.BITS
        h = C.c_void_p()
        check(load().fhe_radix_cast(_ctx().handle, self._h, bits, C.byref(h)))
        return cls._wrap(h, bits)

    @classmethod
    def cast_from(cls, other):
        return other.cast_into(cls)


class FheBool(FheUint):
    BITS = 2


class FheUint8(FheUint):
    BITS = 8


class FheUint32(FheUint):
    BITS = 32


class FheUint64(FheUint):
    BITS = 64


class FheUint128(FheUint):
    BITS = 128


class FheUint256(FheUint):
    BITS = 256


def to_u32_digits(value: int) -> list[int]:
    """num_bigint::BigUint::to_u32_digits: LSB first, no leading zeros, [] for 0."""
    out = []
    while value:
        out.append(value & 0xFFFFFFFF)
        value >>= 32
    return out


class BigUintFHE:
    """src/biguint.rs:8-13 -- Vec<FheUint32> digits, least significant first."""

    def __init__(self, handle):
        self._h = handle

    @property
    def handle(self):
        return self._h

    def __del__(self):
        if getattr(self, "_h", None):
            load().fhe_biguint_destroy(self._h)
            self._h = None

    @classmethod
    def new(cls, value: int, client_key):  # src/biguint.rs:17-31
        limbs = np.array(to_u32_digits(value), dtype=np.uint32)
        h = C.c_void_p()
        check(load().fhe_biguint_encrypt(_ctx().handle, client_key.handle, ptr(limbs, C.c_uint32), limbs.size, C.byref(h)))
        return cls(h)

    def serialize(self) -> bytes:
        return serialize_with(load().fhe_biguint_serialize, _ctx().handle, self._h)

    @classmethod
    def deserialize(cls, data: bytes) -> "BigUintFHE":
        h = C.c_void_p()
        check(load().fhe_biguint_deserialize(_ctx().handle, data, len(data), C.byref(h)))
        return cls(h)

    @classmethod
    def from_u32(cls, value: int, client_key):  # src/biguint.rs:34-36
        return cls.new(value, client_key)

    @classmethod
    def zero(cls, client_key):  # src/biguint.rs:51-53
        return cls.new(0, client_key)

    @classmethod
    def one(cls, client_key):  # src/biguint.rs:56-58
        return cls.new(1, client_key)

    @classmethod
    def from_encrypted_digits(cls, digits):  # src/biguint.rs:46-48
        arr = (C.c_void_p * len(digits))(*[d.handle for d in digits])
        h = C.c_void_p()
        check(load().fhe_biguint_from_digits(arr, len(digits), C.byref(h)))
        return cls(h)

    def __len__(self):
        n = C.c_size_t()
        check(load().fhe_biguint_len(self._h, C.byref(n)))
        return int(n.value)

    @property
    def digits(self):
        out = []
        for i in range(len(self)):
            h = C.c_void_p()
            check(load().fhe_biguint_digit(self._h, i, C.byref(h)))
            out.append(FheUint._wrap(h, 32))
        return out

    @classmethod
    def broadcast(cls, x, root: int = 0, ctx=None):
        """Collective (fhe_ctx_broadcast_biguint): the root's BigUintFHE (e.g. sign_fhe_with_k0's
        encrypted private key, src/schnorr.rs:235) replicated to every rank; other ranks pass None."""
        ctx = ctx or _ctx()
        h = C.c_void_p(_hval(x.handle) if x is not None else None)
        check(load().fhe_ctx_broadcast_biguint(ctx.handle, C.byref(h), root))
        if x is not None and h.value == _hval(x.handle):
            return x
        return cls(h)

    def decrypt_limbs(self, client_key) -> list[int]:
        n = len(self)
        buf = np.zeros(max(n, 1), np.uint32)
        got = C.c_size_t()
        check(load().fhe_biguint_decrypt(_ctx().handle, client_key.handle, self._h, ptr(buf, C.c_uint32), buf.size, C.byref(got)))
        return [int(x) for x in buf[: got.value]]

    def to_biguint(self, client_key) -> int:  # src/biguint.rs:61-76
        return sum(d << (32 * i) for i, d in enumerate(self.decrypt_limbs(client_key)))

    def decrypt_to_u32(self, client_key):  # src/biguint.rs:79-88
        limbs = self.decrypt_limbs(client_key)
        return {0: 0, 1: limbs[0] if limbs else 0}.get(len(limbs))

    def decrypt_to_u64(self, client_key):  # src/biguint.rs:91-105
        limbs = self.decrypt_limbs(client_key)
        if len(limbs) > 2:
            return None
        return sum(d << (32 * i) for i, d in enumerate(limbs))

    def to_radix(self, bits: int):
        """the limbs' blocks as one FheUint of `bits` (concatenation, no bootstrap)"""
        h = C.c_void_p()
        check(load().fhe_biguint_to_radix(self._h, bits, C.byref(h)))
        return FheUint._wrap(h, bits)

    def clone(self):
        h = C.c_void_p()
        check(load().fhe_biguint_clone(self._h, C.byref(h)))
        return BigUintFHE(h)

    def add(self, other, mode: int = COMPAT):
        h = C.c_void_p()
        check(load().fhe_biguint_add(_ctx().handle, self._h, other._h, mode, C.byref(h)))
        return BigUintFHE(h)

    def mul(self, other, mode: int = COMPAT):
        h = C.c_void_p()
        check(load().fhe_biguint_mul(_ctx().handle, self._h, other._h, mode, C.byref(h)))
        return BigUintFHE(h)

    def mul_add(self, other, addend, mode: int = COMPAT):
        """addend + self * other, limbs identical to addend.add(self.mul(other)) (one schedule)"""
        h = C.c_void_p()
        check(load().fhe_biguint_mul_add(_ctx().handle, self._h, other._h, addend._h, mode, C.byref(h)))
        return BigUintFHE(h)

    def mul_add_value(self, other, addend, client_key, mode: int = COMPAT) -> int:
        """the value of mul_add's limbs, computed in column form (fhe_biguint_mul_add_columns: no final
        carry propagation) and decrypted with its carries resolved on the host -- what the signer does"""
        lib = load()
        h = C.c_void_p()
        check(lib.fhe_biguint_mul_add_columns(_ctx().handle, self._h, other._h, addend._h, mode, C.byref(h)))
        try:
            bits = C.c_uint32()
            check(lib.fhe_columns_bits(h, C.byref(bits)))
            n = (bits.value + 63) // 64
            w = np.zeros(n, np.uint64)
            check(lib.fhe_columns_decrypt(_ctx().handle, client_key.handle, h, ptr(w), n))
        finally:
            lib.fhe_columns_destroy(h)
        return sum(int(x) << (64 * i) for i, x in enumerate(w))

    __add__ = add
    __mul__ = mul


LEVEL_SPLIT = 1 << 31  # FHE_LEVEL_SPLIT: the level was fanned out over the ranks


def rank_pbs(ctx) -> int:
    """bootstraps this rank ran itself (fhe_ctx_rank_pbs; emulated ranks: rank 0's share)"""
    v = C.c_uint64()
    check(load().fhe_ctx_rank_pbs(ctx.handle, C.byref(v)))
    return int(v.value)


def level_log(ctx, reset: bool = True) -> list[int]:
    """bootstraps per launched level since the last reset (fhe_ctx_level_log); under fan-out an
    entry carries LEVEL_SPLIT when the level was split over the ranks"""
    n = C.c_size_t()
    check(load().fhe_ctx_level_log(ctx.handle, None, 0, C.byref(n), 0))
    buf = np.zeros(max(1, n.value), np.uint32)
    check(load().fhe_ctx_level_log(ctx.handle, ptr(buf, C.c_uint32), buf.size, C.byref(n), 1 if reset else 0))
    return [int(x) for x in buf[: n.value]]


def stats(ctx):
    p, lv = C.c_uint64(), C.c_uint64()
    check(load().fhe_ctx_stats(ctx.handle, C.byref(p), C.byref(lv)))
    return int(p.value), int(lv.value)
