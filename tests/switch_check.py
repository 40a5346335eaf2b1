"""Every environment switch of INTEGRATION.md 8 gives exact results: the simulated engine (no GPU) runs
BigUintFHE compat / fast products and the radix ops, division included, under the environment it is
started with.  usage: FHE_<SWITCH>=<value> python3 tests/switch_check.py [quick]  (test helper: driven by
test_radix_sim.py::test_environment_switches_simulated)"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in ("oracle", "fhe-sign_amd", "tests"):
    sys.path.insert(0, os.path.join(ROOT, d))
import ref_semantics as R  # noqa: E402
import test_radix_sim as T  # noqa: E402

quick = len(sys.argv) > 1 and sys.argv[1] == "quick"
rng = random.Random(3)
shapes = [(3, 5)] if quick else [(8, 8), (3, 5), (1, 8)]
widths = (32, 128) if quick else (32, 128, 256)
for la, lb in shapes:
    a, b = [rng.getrandbits(32) for _ in range(la)], [rng.getrandbits(32) for _ in range(lb)]
    assert T.sim_mul(a, b, T.COMPAT) == R.biguint_mul(a, b), (la, lb)
    assert R.from_limbs(T.sim_mul(a, b, T.FAST)) == R.from_limbs(a) * R.from_limbs(b), (la, lb)
for bits in widths:
    for op in (T.MUL, T.ADD, T.SUB, T.LT, T.DIV_SCALAR, T.MIN, T.SHR):
        a, b = rng.getrandbits(bits), rng.getrandbits(bits)
        if op == T.SHR:
            b %= bits
        assert T.sim_radix(op, bits, a, b)[0] == T.expect(op, bits, a, b), (op, bits)
    a, b = rng.getrandbits(bits), rng.getrandbits(bits // 2) | 1
    assert T.sim_radix(T.DIVREM, bits, a, b) == (a // b, a % b), bits
print("ok", {k: v for k, v in os.environ.items() if k.startswith("FHE_")})
