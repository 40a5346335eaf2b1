"""Engine graph statistics (FHE_GRAPH_STATS=1, csrc/radix.cpp Engine::graph_stats) of the benchmark ops:
critical-path width per level and two-output blind-rotation candidates (bootstraps sharing their exact
input at input degree <= 7).  usage: FHE_GRAPH_STATS=1 python3 tools/graph_stats.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
os.environ.setdefault("FHE_GRAPH_STATS", "1")
from fhe_sign import (COMPAT, FAST, BigUintFHE, Context, FheUint256, Schnorr, compute_nonce,  # noqa: E402
                      generate_keys, set_server_key)

g = json.load(open(os.path.join(ROOT, "tests", "golden", "biguint_vectors.json")))["mul"][0]
val = lambda limbs: sum(int(x) << (32 * i) for i, x in enumerate(limbs))  # noqa: E731
ck, sk = generate_keys(seed=3)
ctx = Context(0)
ctx.set_server_key(sk)
set_server_key(ctx)
A, B = BigUintFHE.new(val(g["a"]), ck), BigUintFHE.new(val(g["b"]), ck)
for name, fn in (("mul_compat", lambda: A.mul(B, COMPAT)), ("mul_fast", lambda: A.mul(B, FAST))):
    print(f"== {name}", file=sys.stderr, flush=True)
    r = fn()
    ctx.sync()
print("== sign_fhe_with_k0 v0 compat", file=sys.stderr, flush=True)
d, msg = 3, bytes(32)
s = Schnorr()
sig = s.sign_fhe_with_k0(msg, compute_nonce(d, msg, bytes(32)), d, BigUintFHE.new(d, ck), ck, COMPAT)
print("== div256 by encrypted 128-bit", file=sys.stderr, flush=True)
X, D = FheUint256.try_encrypt(val(g["a"]), ck), FheUint256.try_encrypt((1 << 127) | 12345, ck)
q, rm = X.div_rem(D)
ctx.sync()
print("done", file=sys.stderr, flush=True)
