"""fhe_sign -- Python host binding of the MI355X-native TFHE radix engine (fhe-sign_amd).

Mirrors the reference crate's surface (coset-io/fhe-sign):
  generate_keys / set_server_key      tfhe HL API as used at src/schnorr.rs:441-443
  FheUint{8,32,64}                    tfhe FheUint ops used by src/biguint.rs and src/perf_test.rs
  BigUintFHE (+, *)                   src/biguint.rs:8-265
  Schnorr.sign_fhe_with_k0 / sign_fhe src/schnorr.rs:154-290
All ciphertext arithmetic runs on the GPU through lib/libfhe_rocm.so; this package only marshals.
"""
from ._lib import FheError, FheParams, load  # noqa: F401
from .core import (ClientKey, Context, ServerKey, comm_unique_id, default_params, generate_keys,  # noqa: F401
                   multi_bit_params, tuning)
from .integer import (  # noqa: F401,E402
    COMPAT, FAST, PUBLIC, BigUintFHE, FheBool, FheUint, FheUint8, FheUint32, FheUint64, FheUint128, FheUint256, set_server_key,
    LEVEL_SPLIT, level_log, rank_pbs, stats, to_u32_digits)
from .schnorr import Schnorr, compute_nonce, public_key_x  # noqa: F401,E402
