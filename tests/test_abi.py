"""The C-ABI library loads and exports every symbol include/fhe_rocm.h declares (no GPU calls)."""
import ctypes
import os
import re

from conftest import ROOT
from fhe_sign import _lib


def _header_symbols():
    text = open(os.path.join(ROOT, "include", "fhe_rocm.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(fhe_[a-z0-9_]+)\s*\(", text)))


def test_library_loads_and_exports_header_symbols():
    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_binding_covers_header():
    assert sorted(_lib.declared_symbols()) == _header_symbols()


def test_params_default():
    from fhe_sign import default_params
    p = default_params()
    assert (p.lwe_dimension, p.polynomial_size, p.glwe_dimension) == (834, 2048, 1)
    assert (p.pbs_base_log, p.pbs_level, p.ks_base_log, p.ks_level) == (23, 1, 3, 5)
    assert (p.message_modulus, p.carry_modulus) == (4, 4)


def test_no_gpu_context_errors_loudly():
    """Without a GPU the product must refuse, never fall back to CPU arithmetic."""
    import pytest
    from fhe_sign import Context, FheError
    try:
        ctx = Context(0)
    except FheError as e:
        assert "GPU" in str(e) or "hip" in str(e).lower()
        return
    ctx.close()
    pytest.skip("GPU present: nothing to refuse")
