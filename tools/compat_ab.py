"""Same-process A/B of the compat BigUintFHE mul: the carry-count chain (csrc/compat_chain.cpp,
default) against the dependency-wave window adds (FHE_COMPAT_WAVES=1), interleaved rounds; every
result checked against the reference's limb loop (oracle/ref_semantics.py).  Also the 8-limb-key
sign (BIP-340 vector 1: its k + e*d' is an 8 x 8 compat mul-add).
usage: python3 tools/compat_ab.py [rounds]"""
import csv
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ref_semantics as R  # noqa: E402
from fhe_sign import COMPAT, BigUintFHE, Context, Schnorr, compute_nonce, generate_keys, set_server_key, stats  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
ck, sk = generate_keys(seed=0xC0)
ctx = Context(0)
ctx.set_server_key(sk)
set_server_key(ctx)
g = json.load(open(os.path.join(ROOT, "tests", "golden", "biguint_vectors.json")))["mul"][0]
val = lambda limbs: sum(int(x) << (32 * i) for i, x in enumerate(limbs))  # noqa: E731
a, b = val(g["a"]), val(g["b"])
A, B = BigUintFHE.new(a, ck), BigUintFHE.new(b, ck)
ones = (1 << 256) - 1
O1 = BigUintFHE.new(ones, ck)
rows = {r["index"]: r for r in csv.DictReader(open(os.path.join(ROOT, "tests", "golden", "bip340_vectors.csv")))}
r1 = rows["1"]
d1 = int(r1["secret key"], 16)
m1, aux1 = bytes.fromhex(r1["message"]), bytes.fromhex(r1["aux_rand"])
k1 = compute_nonce(d1, m1, aux1)
D1 = BigUintFHE.new(d1, ck)
S = Schnorr()
sig1 = bytes.fromhex(r1["signature"])

cases = [
    ("mul golden", lambda: A.mul(B, COMPAT), lambda r: r.decrypt_limbs(ck) == [int(x) for x in g["out"]]),
    ("mul all-ones (F7)", lambda: O1.mul(O1, COMPAT),
     lambda r: r.decrypt_limbs(ck) == R.biguint_mul(R.to_u32_digits(ones), R.to_u32_digits(ones))),
    ("sign vector 1", lambda: S.sign_fhe_with_k0(m1, k1, d1, D1, ck, COMPAT), lambda r: r == sig1),
]
res = {}
for rnd in range(rounds):
    for variant in ("chain", "waves"):
        if variant == "waves":
            os.environ["FHE_COMPAT_WAVES"] = "1"
        else:
            os.environ.pop("FHE_COMPAT_WAVES", None)
        for name, fn, check in cases:
            fn()  # warm (pools, LUTs)
            ctx.sync()
            p0, l0 = stats(ctx)
            t0 = time.perf_counter()
            r = fn()
            ctx.sync()
            dt = time.perf_counter() - t0
            p1, l1 = stats(ctx)
            ok = check(r)
            res.setdefault((name, variant), []).append(dt)
            print(f"round {rnd} {variant:5s} {name:18s} {dt:.4f} s  {p1 - p0} PBS  {l1 - l0} levels  ok={ok}", flush=True)
            if not ok:
                raise SystemExit(f"MISMATCH {name} {variant}")
for (name, variant), ts in sorted(res.items()):
    print(f"{name:18s} {variant:5s} median {statistics.median(ts):.4f} s  min {min(ts):.4f} s")
