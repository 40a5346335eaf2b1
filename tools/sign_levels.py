"""Level sizes and times of sign_fhe_with_k0 v0 (fused column form and the reference's call site),
classic, with FHE_DEBUG=levels set by the caller (every level synchronised and timed on stderr).
usage: FHE_DEBUG=levels python3 tools/sign_levels.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
from fhe_sign import COMPAT, BigUintFHE, Context, Schnorr, compute_nonce, generate_keys, set_server_key  # noqa: E402

ck, sk = generate_keys(seed=0x5167)
ctx = Context(0)
ctx.set_server_key(sk)
set_server_key(ctx)
d, msg = 3, bytes(32)
k0 = compute_nonce(d, msg, bytes(32))
dF = BigUintFHE.new(d, ck)
s = Schnorr()
ref = s.sign_with_k0(msg, k0, d)
for name, fn in (("fused", lambda: s.sign_fhe_with_k0(msg, k0, d, dF, ck, COMPAT)),
                 ("callsite", lambda: s.sign_fhe_with_k0_callsite(msg, k0, d, dF, ck, COMPAT))):
    fn()
    for rep in range(2):
        print(f"=== {name} rep {rep}", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        r = fn()
        dt = time.perf_counter() - t0
        print(f"=== {name} rep {rep}: {dt * 1e3:.2f} ms ok={r == ref}", file=sys.stderr, flush=True)
t0 = time.perf_counter()
for _ in range(5):
    s.sign_prologue(msg, k0, d)
print(f"prologue (host EC + hash): {(time.perf_counter() - t0) / 5 * 1e3:.2f} ms", file=sys.stderr, flush=True)
t0 = time.perf_counter()
for _ in range(5):
    BigUintFHE.new(k0, ck)
print(f"BigUintFHE::new (8 limbs, host encryption + upload): {(time.perf_counter() - t0) / 5 * 1e3:.2f} ms", file=sys.stderr, flush=True)
ctx.close()
