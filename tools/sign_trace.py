"""sign_fhe_with_k0 (vector 0, compat) under FHE_TRACE_LEVELS: every level synchronised, its size and time,
the host time inside Engine::run between flushes (the products' eager flush runs inside their run() call,
so its level time shows up there in this mode) and any block-pool growth.  usage: python3 tools/sign_trace.py"""
import os, sys, time
os.environ["FHE_TRACE_LEVELS"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fhe-sign_amd"))
from fhe_sign import COMPAT, BigUintFHE, Context, Schnorr, compute_nonce, generate_keys, set_server_key
ck, sk = generate_keys(seed=5)
ctx = Context(0); ctx.set_server_key(sk); set_server_key(ctx)
d, msg = 3, bytes(32)
k0 = compute_nonce(d, msg, bytes(32))
s = Schnorr(); dF = BigUintFHE.new(d, ck); ref = s.sign_with_k0(msg, k0, d)
for i in range(3):
    t0 = time.perf_counter()
    assert s.sign_fhe_with_k0(msg, k0, d, dF, ck, COMPAT) == ref
    print(f"call {i}: {(time.perf_counter() - t0) * 1e3:.2f} ms", file=sys.stderr, flush=True)
