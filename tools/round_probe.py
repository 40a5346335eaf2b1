"""Schedule experiment: wall-clock (median of 3) of the level-bound ops under the level fill granule
FHE_ROUND (env, read by the engine; default 256).  usage: FHE_ROUND=768 python3 tools/round_probe.py"""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
import numpy as np
from fhe_sign import (COMPAT, FAST, BigUintFHE, Context, FheUint256, Schnorr, compute_nonce, generate_keys,
                      level_log, multi_bit_params, set_server_key, stats)

ck, sk = generate_keys(multi_bit_params() if os.environ.get("FHE_PROBE_MB") == "1" else None, seed=9)
ctx = Context(0)
ctx.set_server_key(sk)
set_server_key(ctx)
g = json.load(open(os.path.join(ROOT, "tests", "golden", "biguint_vectors.json")))["mul"][0]
val = lambda l: sum(int(x) << (32 * i) for i, x in enumerate(l))  # noqa: E731
a, b = val(g["a"]), val(g["b"])
A, B = BigUintFHE.new(a, ck), BigUintFHE.new(b, ck)
d, msg = 3, bytes(32)
k0 = compute_nonce(d, msg, bytes(32))
dF = BigUintFHE.new(d, ck)
s = Schnorr()
ref = s.sign_with_k0(msg, k0, d)
A256 = FheUint256.try_encrypt(a, ck)
legs = [("mul_compat", lambda: A.mul(B, COMPAT), lambda r: r.decrypt_limbs(ck) == [int(x) for x in g["out"]]),
        ("mul_fast", lambda: A.mul(B, FAST), lambda r: r.to_biguint(ck) == a * b),
        ("sign_v0", lambda: s.sign_fhe_with_k0(msg, k0, d, dF, ck, COMPAT), lambda r: r == ref),
        ("div_u32", lambda: A256 / 0xDEADBEEF, lambda r: r.decrypt(ck) == a // 0xDEADBEEF)]
A.mul(B, COMPAT).decrypt_limbs(ck)  # warm-up
res = {"round": os.environ.get("FHE_ROUND", "256")}
for name, fn, check in legs:
    ts = []
    level_log(ctx)
    for _ in range(3):
        p0, l0 = stats(ctx)
        t0 = time.perf_counter()
        r = fn()
        ctx.sync()
        ts.append(time.perf_counter() - t0)
        p1, l1 = stats(ctx)
        assert check(r), name
    sizes = level_log(ctx)[-(l1 - l0):]
    hist = {}
    for n in sizes:
        k = "<=256" if n <= 256 else "<=768" if n <= 768 else ">768"
        hist[k] = hist.get(k, 0) + 1
    res[name] = {"s": round(float(np.median(ts)), 4), "pbs": p1 - p0, "levels": l1 - l0, "hist": hist,
                 "big": [n for n in sizes if n > 768]}
print(json.dumps(res), flush=True)
ctx.close()
