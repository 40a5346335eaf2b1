"""ctypes binding of include/fhe_rocm.h (the engine's C ABI).

This is the same binding a maintainer would write for the reference's FFI;
the tests and bench drive the engine exclusively through it.  The shared library must be the
in-tree build (fhe-sign_amd/lib/libfhe_rocm.so); there is no fallback.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# FHE_ROCM_LIB selects another build of the same library (the host-sanitizer build of
# `make -C fhe-sign_amd asan`, tools/sanitize_host.sh); by default the in-tree product build.
LIB_PATH = os.environ.get("FHE_ROCM_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "libfhe_rocm.so")

u8p = C.POINTER(C.c_uint8)
u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)
dblp = C.POINTER(C.c_double)


class FheParams(C.Structure):
    _fields_ = [(name, C.c_uint32) for name in (
        "lwe_dimension", "glwe_dimension", "polynomial_size", "pbs_base_log", "pbs_level",
        "ks_base_log", "ks_level", "lwe_noise_log2", "glwe_noise_log2", "message_modulus",
        "carry_modulus", "grouping")]

    def ggsw_count(self) -> int:
        """GGSWs in the bootstrapping key: n (classic) or (n / g)(2^g - 1) (multi-bit)"""
        g = self.grouping or 1
        return self.lwe_dimension if g == 1 else self.lwe_dimension // g * ((1 << g) - 1)


# fhe_test_transport (include/fhe_rocm.h): the host-staged test hook in place of RCCL
TX_BCAST = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_int)
TX_ALLGATHER = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t)
TX_MIN_U8 = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t)


class TestTransport(C.Structure):
    _fields_ = [("user", C.c_void_p), ("bcast", TX_BCAST), ("allgather", TX_ALLGATHER), ("allreduce_min_u8", TX_MIN_U8)]


# (name, restype, argtypes) -- every symbol include/fhe_rocm.h declares
_SIGNATURES = [
    ("fhe_last_error", C.c_char_p, []),
    ("fhe_params_default", C.c_int, [C.POINTER(FheParams)]),
    ("fhe_params_multi_bit", C.c_int, [C.POINTER(FheParams)]),
    ("fhe_generate_keys", C.c_int, [C.POINTER(FheParams), C.c_uint64, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    ("fhe_generate_keys_device", C.c_int,
     [C.c_void_p, C.POINTER(FheParams), C.c_uint64, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    ("fhe_generate_keys_keyed", C.c_int,
     [C.POINTER(FheParams), C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    ("fhe_generate_keys_device_keyed", C.c_int,
     [C.c_void_p, C.POINTER(FheParams), C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    ("fhe_client_key_destroy", None, [C.c_void_p]),
    ("fhe_server_key_destroy", None, [C.c_void_p]),
    ("fhe_client_key_export", C.c_int, [C.c_void_p, u64p, C.c_size_t, u64p, C.c_size_t]),
    ("fhe_server_key_export", C.c_int, [C.c_void_p, u64p, C.c_size_t, u64p, C.c_size_t]),
    ("fhe_client_key_seed_encryption", C.c_int, [C.c_void_p, C.c_uint64, C.c_uint32]),
    ("fhe_encrypt_block", C.c_int, [C.c_void_p, C.c_uint64, u64p]),
    ("fhe_encrypt_blocks", C.c_int, [C.c_void_p, u64p, C.c_size_t, u64p]),
    ("fhe_decrypt_block", C.c_int, [C.c_void_p, u64p, u64p]),
    ("fhe_ctx_create", C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    ("fhe_ctx_destroy", None, [C.c_void_p]),
    ("fhe_set_server_key", C.c_int, [C.c_void_p, C.c_void_p]),
    ("fhe_ctx_export_fourier_bsk", C.c_int, [C.c_void_p, dblp, C.c_size_t]),
    ("fhe_ctx_sync", C.c_int, [C.c_void_p]),
    ("fhe_lut_register", C.c_int, [C.c_void_p, u32p, C.c_uint32, u32p]),
    ("fhe_pbs_batch", C.c_int, [C.c_void_p, u64p, C.c_size_t, u32p, u64p]),
    ("fhe_pbs_batch_device", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p]),
    ("fhe_device_alloc", C.c_void_p, [C.c_void_p, C.c_size_t]),
    ("fhe_device_free", C.c_int, [C.c_void_p, C.c_void_p]),
    ("fhe_memcpy_h2d", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
    ("fhe_memcpy_d2h", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
    ("fhe_ctx_last_pbs_timing", C.c_int, [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_float)]),
    ("fhe_ctx_enable_timing", C.c_int, [C.c_void_p, C.c_int]),
    ("fhe_ctx_enable_clock", C.c_int, [C.c_void_p, C.c_int]),
    ("fhe_ctx_read_clock", C.c_int, [C.c_void_p, u64p, u64p, u64p]),
    ("fhe_ctx_set_wide_threshold", C.c_int, [C.c_void_p, C.c_int]),
    ("fhe_ctx_set_br_kernel", C.c_int, [C.c_void_p, C.c_int]),
    ("fhe_ctx_set_ks_kernel", C.c_int, [C.c_void_p, C.c_int]),
    ("fhe_comm_unique_id", C.c_int, [C.POINTER(C.c_uint8)]),
    ("fhe_ctx_attach_comm", C.c_int, [C.c_void_p, C.POINTER(C.c_uint8), C.c_int, C.c_int]),
    ("fhe_ctx_attach_comm_timeout", C.c_int, [C.c_void_p, C.POINTER(C.c_uint8), C.c_int, C.c_int, C.c_uint32]),
    ("fhe_ctx_set_comm_timeout", C.c_int, [C.c_void_p, C.c_uint32]),
    ("fhe_ctx_broadcast_server_key", C.c_int, [C.c_void_p, C.c_int]),
    ("fhe_ctx_broadcast_radix", C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.c_int]),
    ("fhe_ctx_broadcast_biguint", C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.c_int]),
    ("fhe_ctx_params", C.c_int, [C.c_void_p, C.POINTER(FheParams)]),
    ("fhe_ctx_detach_comm", C.c_int, [C.c_void_p]),
    ("fhe_ctx_attach_test_transport", C.c_int, [C.c_void_p, C.POINTER(TestTransport), C.c_int, C.c_int]),
    ("fhe_ctx_set_fanout", C.c_int, [C.c_void_p, C.c_uint32, C.c_int]),
    ("fhe_ctx_fanout_info", C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_uint64)]),
    ("fhe_radix_encrypt", C.c_int, [C.c_void_p, C.c_void_p, u64p, C.c_uint32, C.POINTER(C.c_void_p)]),
    ("fhe_radix_trivial", C.c_int, [C.c_void_p, u64p, C.c_uint32, C.POINTER(C.c_void_p)]),
    ("fhe_radix_decrypt", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, u64p, C.c_size_t]),
    ("fhe_radix_num_bits", C.c_int, [C.c_void_p, u32p]),
    ("fhe_radix_clone", C.c_int, [C.c_void_p, C.POINTER(C.c_void_p)]),
    ("fhe_radix_destroy", None, [C.c_void_p]),
    ("fhe_radix_export", C.c_int, [C.c_void_p, C.c_void_p, u64p, C.c_size_t]),
    ("fhe_radix_add", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p)]),
    ("fhe_radix_sub", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p)]),
    ("fhe_radix_mul", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p)]),
    ("fhe_radix_scalar_and", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_void_p)]),
    ("fhe_radix_scalar_shr", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(C.c_void_p)]),
    ("fhe_radix_scalar_shl", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(C.c_void_p)]),
    ("fhe_radix_scalar_add", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_void_p)]),
    ("fhe_radix_scalar_mul", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_void_p)]),
    ("fhe_radix_scalar_div", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_void_p)]),
    ("fhe_radix_scalar_rem", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_void_p)]),
    ("fhe_client_key_params", C.c_int, [C.c_void_p, C.c_void_p]),
    ("fhe_server_key_params", C.c_int, [C.c_void_p, C.c_void_p]),
    ("fhe_client_key_serialize", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    ("fhe_client_key_deserialize", C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p)]),
    ("fhe_server_key_serialize", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    ("fhe_server_key_deserialize", C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p)]),
    ("fhe_radix_serialize", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    ("fhe_radix_deserialize", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p)]),
    ("fhe_biguint_serialize", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    ("fhe_biguint_deserialize", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p)]),
    ("fhe_radix_div", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p)]),
    ("fhe_radix_rem", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p)]),
    ("fhe_radix_divrem", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    ("fhe_radix_scalar_and_words", C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t, C.POINTER(C.c_void_p)]),
    ("fhe_radix_scalar_add_words", C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t, C.POINTER(C.c_void_p)]),
    ("fhe_radix_scalar_mul_words", C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t, C.POINTER(C.c_void_p)]),
    ("fhe_radix_scalar_mul_add_words", C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t,
                                                C.POINTER(C.c_uint64), C.c_size_t, C.POINTER(C.c_void_p)]),
    ("fhe_radix_scalar_div_words", C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t, C.POINTER(C.c_void_p)]),
    ("fhe_radix_scalar_rem_words", C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t, C.POINTER(C.c_void_p)]),
    ("fhe_radix_cast", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(C.c_void_p)]),
    ("fhe_radix_min", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p)]),
    ("fhe_radix_max", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p)]),
    ("fhe_radix_lt", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p)]),
    ("fhe_radix_shr", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p)]),
    ("fhe_radix_shl", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p)]),
    ("fhe_radix_bitand", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p)]),
    ("fhe_ctx_stats", C.c_int, [C.c_void_p, u64p, u64p]),
    ("fhe_ctx_level_log", C.c_int, [C.c_void_p, u32p, C.c_size_t, C.POINTER(C.c_size_t), C.c_int]),
    ("fhe_ctx_rank_pbs", C.c_int, [C.c_void_p, u64p]),
    ("fhe_schedule_levels", C.c_int, [C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.c_size_t, C.c_int,
                                      C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    ("fhe_schedule_levels_ranks", C.c_int, [C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.c_size_t, C.c_int, C.c_int,
                                            C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    ("fhe_progress_marks_probe", C.c_int, [C.c_uint32, u32p]),
    ("fhe_host_biguint_mul", C.c_int, [u32p, C.c_size_t, u32p, C.c_size_t, u32p, C.c_size_t, C.c_int, u32p, C.c_size_t,
                                       C.POINTER(C.c_size_t)]),
    ("fhe_host_biguint_mul_fingerprint", C.c_int, [C.c_size_t, C.c_size_t, C.c_size_t, C.c_int,
                                                   C.POINTER(C.c_uint64)]),
    ("fhe_host_set_tuning", C.c_int, [C.c_int, C.c_int64, C.POINTER(C.c_int64)]),
    ("fhe_host_biguint_mul_stats", C.c_int, [C.c_size_t, C.c_size_t, C.c_size_t, C.c_int, C.POINTER(C.c_uint64),
                                             C.POINTER(C.c_uint64), u32p, C.c_size_t]),
    ("fhe_host_radix_stats", C.c_int, [C.c_int, C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), u32p,
                                       C.c_size_t]),
    ("fhe_host_sim_biguint_mul", C.c_int, [u32p, C.c_size_t, u32p, C.c_size_t, u32p, C.c_size_t, C.c_int, u32p,
                                           C.c_size_t, C.POINTER(C.c_size_t), C.POINTER(C.c_uint64),
                                           C.POINTER(C.c_uint64)]),
    ("fhe_host_sim_radix", C.c_int, [C.c_int, C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                     C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                     C.POINTER(C.c_uint64)]),
    ("fhe_host_sim_biguint_mul_add_columns", C.c_int, [u32p, C.c_size_t, u32p, C.c_size_t, u32p, C.c_size_t, C.c_int,
                                                       C.POINTER(C.c_uint64), C.c_size_t, u32p, C.POINTER(C.c_uint64),
                                                       C.POINTER(C.c_uint64)]),
    ("fhe_host_sim_chain_g", C.c_int, [u8p, C.c_size_t, u32p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("fhe_biguint_mul_add_columns", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                              C.POINTER(C.c_void_p)]),
    ("fhe_radix_scalar_mul_add_columns", C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t,
                                                   C.POINTER(C.c_uint64), C.c_size_t, C.POINTER(C.c_void_p)]),
    ("fhe_columns_bits", C.c_int, [C.c_void_p, u32p]),
    ("fhe_columns_decrypt", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t]),
    ("fhe_columns_destroy", None, [C.c_void_p]),
    ("fhe_biguint_encrypt", C.c_int, [C.c_void_p, C.c_void_p, u32p, C.c_size_t, C.POINTER(C.c_void_p)]),
    ("fhe_biguint_from_digits", C.c_int, [C.POINTER(C.c_void_p), C.c_size_t, C.POINTER(C.c_void_p)]),
    ("fhe_biguint_decrypt", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, u32p, C.c_size_t, C.POINTER(C.c_size_t)]),
    ("fhe_biguint_len", C.c_int, [C.c_void_p, C.POINTER(C.c_size_t)]),
    ("fhe_biguint_digit", C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p)]),
    ("fhe_biguint_to_radix", C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_void_p)]),
    ("fhe_biguint_clone", C.c_int, [C.c_void_p, C.POINTER(C.c_void_p)]),
    ("fhe_biguint_destroy", None, [C.c_void_p]),
    ("fhe_biguint_add", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]),
    ("fhe_biguint_mul", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]),
    ("fhe_biguint_mul_add", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]),
    ("fhe_schnorr_public_key", C.c_int, [u8p, u8p]),
    ("fhe_schnorr_compute_nonce", C.c_int, [u8p, u8p, C.c_size_t, u8p, u8p]),
    ("fhe_schnorr_sign_with_k0", C.c_int, [u8p, C.c_size_t, u8p, u8p, u8p]),
    ("fhe_schnorr_sign", C.c_int, [u8p, C.c_size_t, u8p, u8p, u8p]),
    ("fhe_schnorr_sign_prologue", C.c_int, [u8p, C.c_size_t, u8p, u8p, u8p, u8p, u8p]),
    ("fhe_schnorr_sign_fhe_with_k0", C.c_int, [C.c_void_p, C.c_void_p, u8p, C.c_size_t, u8p, u8p, C.c_void_p, C.c_int, u8p]),
    ("fhe_schnorr_sign_fhe_with_k0_batch", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p),
                                                    C.POINTER(C.c_size_t), C.c_char_p, C.c_char_p,
                                                    C.POINTER(C.c_void_p), C.c_int, C.c_char_p]),
    ("fhe_schnorr_sign_fhe", C.c_int, [C.c_void_p, C.c_void_p, u8p, C.c_size_t, u8p, u8p, C.c_int, u8p]),
    ("fhe_schnorr_verify", C.c_int, [u8p, C.c_size_t, u8p, C.c_size_t, u8p, C.c_size_t]),
]

_lib = None


class FheError(RuntimeError):
    """a negative status of the C ABI; `code` is the FHE_ERR_* value"""

    def __init__(self, msg: str, code: int = 0):
        super().__init__(msg)
        self.code = code


FHE_ERR_TIMEOUT = -6


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FheError(f"native engine not built: {LIB_PATH} missing (run __graft_entry__.build())")
    lib = C.CDLL(LIB_PATH)
    for name, res, args in _SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def declared_symbols() -> list[str]:
    return [s[0] for s in _SIGNATURES]


def check(rc: int) -> None:
    if rc != 0:
        msg = load().fhe_last_error()
        raise FheError(f"fhe error {rc}: {msg.decode() if msg else ''}", rc)


def ptr(arr, ctype=C.c_uint64):
    """Pointer to a contiguous numpy array."""
    return arr.ctypes.data_as(C.POINTER(ctype))


def serialize_with(fn, *args) -> bytes:
    """size query (NULL buffer), then fill: the C ABI's serialization convention"""
    n = C.c_size_t(0)
    check(fn(*args, None, 0, C.byref(n)))
    buf = (C.c_uint8 * n.value)()
    check(fn(*args, buf, n.value, C.byref(n)))
    return bytes(buf)
