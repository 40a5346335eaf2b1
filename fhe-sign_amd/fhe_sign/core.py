"""Keys, device context and the raw PBS boundary (thin wrappers over the C ABI)."""
from __future__ import annotations

import contextlib
import ctypes as C

import numpy as np

from ._lib import FheParams, check, load, ptr, serialize_with

BIG_CT = 2049  # big LWE ciphertext words


def default_params() -> FheParams:
    p = FheParams()
    check(load().fhe_params_default(C.byref(p)))
    return p


def multi_bit_params() -> FheParams:
    """default parameters with the multi-bit blind rotation (grouping 2; fhe_params.grouping)"""
    p = FheParams()
    check(load().fhe_params_multi_bit(C.byref(p)))
    return p


class ClientKey:
    def __init__(self, handle, params: FheParams):
        self._h = handle
        self.params = params

    @property
    def handle(self):
        return self._h

    def __del__(self):
        if getattr(self, "_h", None):
            load().fhe_client_key_destroy(self._h)
            self._h = None

    def export(self):
        n = self.params.lwe_dimension
        lwe = np.zeros(n, np.uint64)
        glwe = np.zeros(self.params.polynomial_size, np.uint64)
        check(load().fhe_client_key_export(self._h, ptr(lwe), n, ptr(glwe), glwe.size))
        return lwe, glwe

    def serialize(self) -> bytes:
        """own versioned format (include/fhe_rocm.h, serial.h), encryption-stream state included"""
        return serialize_with(load().fhe_client_key_serialize, self._h)

    @classmethod
    def deserialize(cls, data: bytes) -> "ClientKey":
        h = C.c_void_p()
        check(load().fhe_client_key_deserialize(data, len(data), C.byref(h)))
        p = FheParams()
        check(load().fhe_client_key_params(h, C.byref(p)))
        return cls(h, p)

    def seed_encryption(self, seed: int, stream: int = 100) -> None:
        check(load().fhe_client_key_seed_encryption(self._h, seed, stream))

    def encrypt_block(self, value: int) -> np.ndarray:
        ct = np.zeros(BIG_CT, np.uint64)
        check(load().fhe_encrypt_block(self._h, value, ptr(ct)))
        return ct

    def encrypt_blocks(self, values) -> np.ndarray:
        """many blocks at once: identical to encrypt_block in a loop (multi-threaded on the host)"""
        v = np.ascontiguousarray(np.asarray(values, dtype=np.uint64))
        out = np.zeros((v.size, BIG_CT), np.uint64)
        check(load().fhe_encrypt_blocks(self._h, ptr(v), v.size, ptr(out)))
        return out

    def decrypt_block(self, ct: np.ndarray) -> int:
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        out = C.c_uint64(0)
        check(load().fhe_decrypt_block(self._h, ptr(ct), C.byref(out)))
        return int(out.value)


class ServerKey:
    def __init__(self, handle, params: FheParams):
        self._h = handle
        self.params = params

    @property
    def handle(self):
        return self._h

    def __del__(self):
        if getattr(self, "_h", None):
            load().fhe_server_key_destroy(self._h)
            self._h = None

    def serialize(self) -> bytes:
        return serialize_with(load().fhe_server_key_serialize, self._h)

    @classmethod
    def deserialize(cls, data: bytes) -> "ServerKey":
        h = C.c_void_p()
        check(load().fhe_server_key_deserialize(data, len(data), C.byref(h)))
        p = FheParams()
        check(load().fhe_server_key_params(h, C.byref(p)))
        return cls(h, p)

    def export(self):
        p = self.params
        n, N, L = p.lwe_dimension, p.polynomial_size, p.ks_level
        ksk = np.zeros(N * L * (n + 1), np.uint64)
        bsk = np.zeros(p.ggsw_count() * 4 * N, np.uint64)
        check(load().fhe_server_key_export(self._h, ptr(ksk), ksk.size, ptr(bsk), bsk.size))
        return ksk, bsk


def comm_unique_id() -> bytes:
    """RCCL unique id (rank 0 creates it and shares it out of band, e.g. over torch.distributed)."""
    buf = (C.c_uint8 * 128)()
    check(load().fhe_comm_unique_id(buf))
    return bytes(buf)


def generate_keys(params: FheParams | None = None, seed: int | None = None, device: "Context | None" = None):
    """tfhe::generate_keys(ConfigBuilder::default().build()) -- src/schnorr.rs:441-442.

    seed=None (the default) keys every ChaCha20 stream with 32 bytes from os.urandom, as tfhe-rs
    draws from the OS CSPRNG.  An integer seed gives DETERMINISTIC, INSECURE keys (a public
    expansion of 64 bits) for tests and golden vectors only.
    With `device` (a Context), the server key is generated on that GPU: identical key words
    (fhe_generate_keys_device*); the key is returned, not installed."""
    import os

    p = params or default_params()
    ck, sk = C.c_void_p(), C.c_void_p()
    lib = load()
    if seed is None:
        key = (C.c_uint8 * 32).from_buffer_copy(os.urandom(32))
        if device is None:
            check(lib.fhe_generate_keys_keyed(C.byref(p), key, C.byref(ck), C.byref(sk)))
        else:
            check(lib.fhe_generate_keys_device_keyed(device.handle, C.byref(p), key, C.byref(ck), C.byref(sk)))
        C.memset(key, 0, 32)
    elif device is None:
        check(lib.fhe_generate_keys(C.byref(p), seed, C.byref(ck), C.byref(sk)))
    else:
        check(lib.fhe_generate_keys_device(device.handle, C.byref(p), seed, C.byref(ck), C.byref(sk)))
    return ClientKey(ck, p), ServerKey(sk, p)


class Context:
    """One GPU + installed server key (tfhe::set_server_key, src/schnorr.rs:443)."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        check(load().fhe_ctx_create(device, C.byref(h)))
        self._h = h
        self.params = None

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None):
            load().fhe_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def set_server_key(self, sk: ServerKey) -> None:
        check(load().fhe_set_server_key(self._h, sk.handle))
        self.params = sk.params

    def export_fourier_bsk(self) -> np.ndarray:
        out = np.zeros(self.params.ggsw_count() * 4 * 1024 * 2, np.float64)
        check(load().fhe_ctx_export_fourier_bsk(self._h, ptr(out, C.c_double), out.size))
        return out

    def lut(self, table) -> int:
        t = np.ascontiguousarray(np.asarray(table, dtype=np.uint32))
        out = C.c_uint32(0)
        check(load().fhe_lut_register(self._h, ptr(t, C.c_uint32), t.size, C.byref(out)))
        return int(out.value)

    def pbs(self, cts: np.ndarray, lut_ids) -> np.ndarray:
        cts = np.ascontiguousarray(cts, dtype=np.uint64).reshape(-1, BIG_CT)
        ids = np.ascontiguousarray(np.broadcast_to(np.asarray(lut_ids, np.uint32), (cts.shape[0],)))
        out = np.zeros_like(cts)
        check(load().fhe_pbs_batch(self._h, ptr(cts), cts.shape[0], ptr(ids, C.c_uint32), ptr(out)))
        return out

    # device-resident helpers (bench)
    def alloc(self, nbytes: int) -> int:
        p = load().fhe_device_alloc(self._h, nbytes)
        if not p:
            check(-4)
        return p

    def free(self, p: int) -> None:
        check(load().fhe_device_free(self._h, C.c_void_p(p)))

    def h2d(self, dst: int, arr: np.ndarray) -> None:
        check(load().fhe_memcpy_h2d(self._h, C.c_void_p(dst), arr.ctypes.data_as(C.c_void_p), arr.nbytes))

    def d2h(self, arr: np.ndarray, src: int) -> None:
        check(load().fhe_memcpy_d2h(self._h, arr.ctypes.data_as(C.c_void_p), C.c_void_p(src), arr.nbytes))

    def pbs_device(self, d_in: int, count: int, d_lut: int, d_out: int) -> None:
        check(load().fhe_pbs_batch_device(self._h, C.c_void_p(d_in), count, C.c_void_p(d_lut), C.c_void_p(d_out)))

    def sync(self) -> None:
        check(load().fhe_ctx_sync(self._h))

    def set_br_kernel(self, kind: int) -> None:
        """4 = br_qy.hip, the throughput kernel (classic and multi-bit); the retired kernels 0 (2-wave), 1 (quad),
        2 (pair) and 3 (qx) are refused (FHE_ERR_INVALID)."""
        check(load().fhe_ctx_set_br_kernel(self._h, int(kind)))

    def set_ks_kernel(self, kind: int) -> None:
        """0 = 64-bit VALU keyswitch, 1 = int8 matrix-core keyswitch (default); identical results"""
        check(load().fhe_ctx_set_ks_kernel(self._h, int(kind)))

    def set_wide_threshold(self, threshold: int) -> None:
        check(load().fhe_ctx_set_wide_threshold(self._h, int(threshold)))

    # ---- multi-GPU fan-out (one process per GPU)
    def attach_comm(self, unique_id: bytes, nranks: int, rank: int, timeout_ms: int = 120000) -> None:
        """non-blocking RCCL init polled against `timeout_ms`: a peer that never joins gives an error
        (FHE_ERR_TIMEOUT), not a hang"""
        buf = (C.c_uint8 * 128).from_buffer_copy(unique_id)
        check(load().fhe_ctx_attach_comm_timeout(self._h, buf, nranks, rank, int(timeout_ms)))

    def set_comm_timeout(self, timeout_ms: int) -> None:
        """the attached communicator's deadline: time a bounded wait may pass without progress"""
        check(load().fhe_ctx_set_comm_timeout(self._h, int(timeout_ms)))

    def ready(self) -> bool:
        """the context exists and its device is usable (checked before any collective is entered)"""
        return bool(getattr(self, "_h", None)) and load().fhe_ctx_sync(self._h) == 0

    def broadcast_server_key(self, root: int = 0) -> None:
        """collective: replicate rank `root`'s installed server key to every rank (RCCL)"""
        check(load().fhe_ctx_broadcast_server_key(self._h, int(root)))
        p = FheParams()
        check(load().fhe_ctx_params(self._h, C.byref(p)))
        self.params = p

    def detach_comm(self) -> None:
        check(load().fhe_ctx_detach_comm(self._h))

    def set_fanout(self, min_level: int = 257, emulate_ranks: int = 0) -> None:
        check(load().fhe_ctx_set_fanout(self._h, int(min_level), int(emulate_ranks)))

    def fanout_info(self):
        r, n, lv = C.c_int(), C.c_int(), C.c_uint64()
        check(load().fhe_ctx_fanout_info(self._h, C.byref(r), C.byref(n), C.byref(lv)))
        return int(r.value), int(n.value), int(lv.value)

    def enable_timing(self, on: bool = True) -> None:
        check(load().fhe_ctx_enable_timing(self._h, 1 if on else 0))

    def last_pbs_timing(self):
        ks, br = C.c_float(), C.c_float()
        check(load().fhe_ctx_last_pbs_timing(self._h, C.byref(ks), C.byref(br)))
        return float(ks.value), float(br.value)

    def enable_clock(self, on: bool = True) -> None:
        """clock probe of the throughput blind rotate (fhe_ctx_enable_clock); enabling resets its sums"""
        check(load().fhe_ctx_enable_clock(self._h, 1 if on else 0))

    def read_clock(self):
        """(shader cycles, 100 MHz ticks, workgroups) summed over the probed launches' workgroups"""
        cy, tk, wg = C.c_uint64(), C.c_uint64(), C.c_uint64()
        check(load().fhe_ctx_read_clock(self._h, C.byref(cy), C.byref(tk), C.byref(wg)))
        return int(cy.value), int(tk.value), int(wg.value)


TUNE_KEYS = {"kara_min": 1, "kara_compat_min": 2, "kara_force": 3, "div_r16_lead": 4, "scalar_div_residue": 5,
             "flush_depth": 6}


@contextlib.contextmanager
def tuning(**values):
    """Test hook (fhe_host_set_tuning): move the radix algorithms' size rules for the duration of a
    with-block -- e.g. tuning(kara_min=6) -- and restore them after.  Process-wide."""
    old = {}
    try:
        for k, v in values.items():
            prev = C.c_int64()
            check(load().fhe_host_set_tuning(TUNE_KEYS[k], int(v), C.byref(prev)))
            old[k] = prev.value
        yield
    finally:
        for k, v in old.items():
            check(load().fhe_host_set_tuning(TUNE_KEYS[k], v, None))
