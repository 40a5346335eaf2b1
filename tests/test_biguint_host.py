"""BigUintFHE mul / mul-add limb algorithms on the CPU (no GPU): publicly known limbs through the
engine's host folding (fhe_host_biguint_mul -> Engine host_only), the same radix code path the GPU
runs, every lookup evaluated on the host.  Checked against oracle/ref_semantics.py (the reference's
limb loop, src/biguint.rs:194-265, lost carries included) -- in particular the compat carry-count
chain (csrc/compat_chain.cpp) on inputs that make the reference drop carries."""
import ctypes
import random

import pytest

import ref_semantics as R
from fhe_sign import _lib, tuning

M = 1 << 32
COMPAT, FAST = 0, 1


def host_mul(a, b, mode, k=None):
    A = (ctypes.c_uint32 * max(1, len(a)))(*a)
    B = (ctypes.c_uint32 * max(1, len(b)))(*b)
    K = (ctypes.c_uint32 * max(1, len(k)))(*k) if k is not None else None
    cap = len(a) + len(b) + (len(k) if k else 0) + 2
    out = (ctypes.c_uint32 * cap)()
    n = ctypes.c_size_t()
    kp = ctypes.cast(K, ctypes.POINTER(ctypes.c_uint32)) if K is not None else None
    rc = _lib.load().fhe_host_biguint_mul(A, len(a), B, len(b), kp, len(k) if k else 0, mode, out, cap,
                                          ctypes.byref(n))
    assert rc == 0, _lib.load().fhe_last_error()
    return list(out[: n.value])


def _cases(seed, count):
    rng = random.Random(seed)
    special = [0, 1, M - 1, M - 2, M // 2, 0xFFFF0000, M - 16, M - 17, 15, 16]
    for t in range(count):
        la, lb = rng.randint(2, 8), rng.randint(2, 8)
        kind = t % 3
        if kind == 0:
            a, b = [rng.getrandbits(32) for _ in range(la)], [rng.getrandbits(32) for _ in range(lb)]
        elif kind == 1:
            a, b = [rng.choice(special) for _ in range(la)], [rng.choice(special) for _ in range(lb)]
        else:
            a = [rng.choice((M - 1, M - 2, rng.getrandbits(32))) for _ in range(la)]
            b = [rng.choice((M - 1, 1, rng.getrandbits(32))) for _ in range(lb)]
        yield a, b


def test_compat_chain_matches_reference_limb_loop():
    drops = 0
    for a, b in _cases(11, 60):
        want = R.biguint_mul(a, b)
        drops += R.from_limbs(want) != R.from_limbs(a) * R.from_limbs(b)
        assert host_mul(a, b, COMPAT) == want, (a, b)
    assert drops >= 5  # the set exercises the reference's lost carries


def test_compat_chain_8x8_all_ones_and_golden():
    ones = [M - 1] * 8
    assert host_mul(ones, ones, COMPAT) == R.biguint_mul(ones, ones)
    import json
    import os
    from conftest import ROOT
    for g in json.load(open(os.path.join(ROOT, "tests", "golden", "biguint_vectors.json")))["mul"]:
        if min(len(g["a"]), len(g["b"])) >= 2:
            assert host_mul([int(x) for x in g["a"]], [int(x) for x in g["b"]], COMPAT) == [int(x) for x in g["out"]]


@pytest.mark.parametrize("la,lb", [(1, 8), (8, 1), (2, 2), (8, 12), (3, 7)])
def test_compat_shapes(la, lb):
    rng = random.Random(la * 31 + lb)
    a = [rng.choice((M - 1, rng.getrandbits(32))) for _ in range(la)]
    b = [rng.choice((M - 1, rng.getrandbits(32))) for _ in range(lb)]
    assert host_mul(a, b, COMPAT) == R.biguint_mul(a, b)


def test_fast_and_mul_add():
    rng = random.Random(3)
    for _ in range(6):
        a = [rng.getrandbits(32) for _ in range(8)]
        b = [rng.choice((M - 1, rng.getrandbits(32))) for _ in range(8)]
        k = [rng.getrandbits(32) for _ in range(8)]
        assert R.from_limbs(host_mul(a, b, FAST)) == R.from_limbs(a) * R.from_limbs(b)
        assert host_mul(a, b, COMPAT, k) == R.biguint_add(k, R.biguint_mul(a, b))


@pytest.mark.parametrize("kmin", [6, 7, 16])
def test_karatsuba_split_algebra(kmin):
    """The Karatsuba split of full products (csrc/radix.cpp mul_problems_ops) forced onto publicly known
    operands (tuning kara_force): its offsets, complements and public constants, recursion down to kmin
    blocks (at least 6), odd halves and trimmed zero tops, against the reference limb loop in both modes."""
    with tuning(kara_force=1, kara_min=kmin):
        _karatsuba_cases(kmin)


def _karatsuba_cases(kmin):
    for a, b in _cases(77 + kmin, 12):
        assert R.from_limbs(host_mul(a, b, FAST)) == R.from_limbs(a) * R.from_limbs(b)
        assert host_mul(a, b, COMPAT) == R.biguint_mul(a, b)
    full = [M - 1] * 8
    assert R.from_limbs(host_mul(full, full, FAST)) == R.from_limbs(full) ** 2
    assert host_mul(full, full, COMPAT) == R.biguint_mul(full, full)
    k = [M - 1, 3, 0, M - 2]
    assert host_mul(full, full, COMPAT, k) == R.biguint_add(k, R.biguint_mul(full, full))
    assert R.from_limbs(host_mul(full, full, FAST, k)) == R.from_limbs(full) ** 2 + R.from_limbs(k)
