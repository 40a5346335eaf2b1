"""Schedule budgets of the hot-path ops (dry engine, no GPU): the bootstraps and launch levels each op is
scheduled into (fhe_host_radix_stats / fhe_host_biguint_mul_stats) may not grow past the round-5
figures -- the op latencies on the GPU follow the level counts (one latency round of ~2.0-2.4 ms each,
DESIGN.md 5-6), so a change that adds levels shows up here before any GPU run.  Budgets carry a small
margin over the measured schedule; lowering one when an op improves is the intended maintenance."""
import ctypes as C

import pytest

from fhe_sign import _lib

DIVREM, MUL, ADD, SUB, SHR, LT, DIV_SCALAR = range(7)
COMPAT, FAST = 0, 1
STATS_COLUMNS = 0x100  # FHE_HOST_STATS_COLUMNS


def radix_stats(op, bits):
    p, lev = C.c_uint64(), C.c_uint64()
    lib = _lib.load()
    assert lib.fhe_host_radix_stats(op, bits, C.byref(p), C.byref(lev), None, 0) == 0, lib.fhe_last_error()
    return p.value, lev.value


def mul_stats(la, lb, lk, mode):
    p, lev = C.c_uint64(), C.c_uint64()
    lib = _lib.load()
    assert lib.fhe_host_biguint_mul_stats(la, lb, lk, mode, C.byref(p), C.byref(lev), None, 0) == 0, \
        lib.fhe_last_error()
    return p.value, lev.value


# (op, bits): (max bootstraps, max levels) -- measured r5: 139,578/660 (32 leading radix-16 blocks),
# 26,166/14, 624/7, 624/7, 2,050/6, 193/6 (strict comparison, no negation level), 8,309/17 (residue split; 14,541/13 by the multiplier) at 256
# bits; the 32-bit division trades bootstraps
# for levels (5,444/43 against 1,997/75 radix-4 only)
RADIX_BUDGET = {
    (DIVREM, 256): (141_000, 660), (DIVREM, 32): (5_600, 43),
    (MUL, 256): (26_700, 14), (ADD, 256): (640, 7), (SUB, 256): (640, 7),
    (SHR, 256): (2_100, 6), (SHR, 32): (180, 5), (LT, 256): (200, 6), (DIV_SCALAR, 256): (8_500, 17),
}


@pytest.mark.parametrize("key", sorted(RADIX_BUDGET))
def test_radix_op_schedule_budget(key):
    pbs, levels = radix_stats(*key)
    max_pbs, max_levels = RADIX_BUDGET[key]
    assert levels <= max_levels and pbs <= max_pbs, (key, pbs, levels)


def test_biguint_mul_schedule_budget():
    """256-bit BigUintFHE mul: compat (the reference's limbs, carry-count chain, Karatsuba limb products)
    and fast (true product, Karatsuba twice): r5 57,564 PBS / 44 levels and 29,816 / 29; r6 59,020 / 44 for
    compat (the chain's carry-aware near indicators, compat_chain_g: +13 bootstraps per prefix)."""
    pbs, levels = mul_stats(8, 8, 0, COMPAT)
    assert levels <= 44 and pbs <= 59_100, (pbs, levels)
    pbs, levels = mul_stats(8, 8, 0, FAST)
    assert levels <= 29 and pbs <= 30_300, (pbs, levels)


def test_signer_column_form_schedule_budget():
    """sign_fhe_with_k0's FHE block k + e*d' on vector 0's shape (8 x 1 limbs + 8): the column form the
    signer uses (FHE_HOST_STATS_COLUMNS: biguint_mul_add_columns) against the normalized mul-add of the
    reference's call site."""
    pbs, levels = mul_stats(8, 1, 8, COMPAT | STATS_COLUMNS)
    assert levels <= 4 and pbs <= 6_200, (pbs, levels)  # r6: 6,132 (first compression round capped)
    pbs_n, levels_n = mul_stats(8, 1, 8, COMPAT)
    assert levels_n > levels and pbs_n > pbs
