"""Wall-clock of the reference-level operations (configs 2-4) with engine statistics.
usage: python3 tools/ops_timing.py [package_dir]   (package_dir: a build_variants/NAME copy; default
the in-tree fhe-sign_amd package)"""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.abspath(sys.argv[1]) if len(sys.argv) > 1 else os.path.join(ROOT, "fhe-sign_amd")
sys.path.insert(0, PKG); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import random
import ref_semantics as R
from fhe_sign import *
from fhe_sign import stats

ck, sk = generate_keys(seed=9)
ctx = Context(0); ctx.set_server_key(sk); set_server_key(ctx)
rng = random.Random(0xF11E51)
out = {}
def timed(name, fn, check=None):
    p0, l0 = stats(ctx); t0 = time.perf_counter(); r = fn(); ctx.sync(); dt = time.perf_counter() - t0
    p1, l1 = stats(ctx)
    ok = check(r) if check else None
    out[name] = {"s": round(dt, 4), "pbs": p1 - p0, "levels": l1 - l0, "pbs_per_s": round((p1 - p0) / dt), "ok": ok}
    print(name, out[name], flush=True)
    return r
a, b = rng.getrandbits(256) | 1 << 255, rng.getrandbits(256) | 1 << 255
A, B = BigUintFHE.new(a, ck), BigUintFHE.new(b, ck)
timed("warmup_add", lambda: A.add(B, FAST))
timed("biguint256_add_compat", lambda: A.add(B, COMPAT), lambda r: r.to_biguint(ck) == a + b)
timed("biguint256_add_fast", lambda: A.add(B, FAST), lambda r: r.to_biguint(ck) == a + b)
timed("biguint256_mul_compat", lambda: A.mul(B, COMPAT), lambda r: r.decrypt_limbs(ck) == R.biguint_mul(R.to_u32_digits(a), R.to_u32_digits(b)))
timed("biguint256_mul_fast", lambda: A.mul(B, FAST), lambda r: r.to_biguint(ck) == a * b)
x = rng.getrandbits(32)
X = FheUint32.try_encrypt(x, ck)
timed("fheuint32_div5", lambda: X / 5, lambda r: r.decrypt(ck) == x // 5)
timed("fheuint32_mul", lambda: X * X, lambda r: r.decrypt(ck) == (x * x) % 2**32)
timed("fheuint32_add", lambda: X + X, lambda r: r.decrypt(ck) == (2 * x) % 2**32)
timed("fheuint32_shr_enc", lambda: X >> FheUint32.try_encrypt(13, ck), lambda r: r.decrypt(ck) == x >> 13)
y = rng.getrandbits(256)
Y = FheUint64.try_encrypt(y % 2**64, ck)
timed("fheuint64_div_random", lambda: Y / 0xDEADBEEF, lambda r: r.decrypt(ck) == (y % 2**64) // 0xDEADBEEF)
Z = FheUint64.try_encrypt(0xDEADBEEF12345, ck)
timed("fheuint64_div_encrypted", lambda: Y.div_rem(Z), lambda r: (r[0].decrypt(ck), r[1].decrypt(ck)) == divmod(y % 2**64, 0xDEADBEEF12345))
A256, D256 = FheUint256.try_encrypt(a, ck), FheUint256.try_encrypt(b >> 128, ck)
timed("div256_by_encrypted", lambda: A256.div_rem(D256), lambda r: (r[0].decrypt(ck), r[1].decrypt(ck)) == divmod(a, b >> 128))
d = 3; msg = bytes(32); k0 = compute_nonce(d, msg, bytes(32)); dF = BigUintFHE.new(d, ck)
s = Schnorr()
timed("sign_fhe_with_k0_v0_compat", lambda: s.sign_fhe_with_k0(msg, k0, d, dF, ck, COMPAT), lambda r: r == s.sign_with_k0(msg, k0, d))
timed("sign_fhe_with_k0_v0_fast", lambda: s.sign_fhe_with_k0(msg, k0, d, dF, ck, FAST), lambda r: r == s.sign_with_k0(msg, k0, d))
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "ops_timing.json"), "w"), indent=1)
