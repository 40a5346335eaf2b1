"""Where the time of sign_fhe_with_k0 (BIP-340 vector 0) goes on the GPU box: host encryption of the
two 8-limb operands (e_fhe, k_fhe: 128 blocks each) and their upload, against the whole call.
usage: python3 tools/sign_probe.py"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
import numpy as np  # noqa: E402
from fhe_sign import COMPAT, BigUintFHE, Context, Schnorr, compute_nonce, generate_keys, set_server_key  # noqa: E402

ck, sk = generate_keys(seed=5)
ctx = Context(0)
ctx.set_server_key(sk)
set_server_key(ctx)
d, msg = 3, bytes(32)
k0 = compute_nonce(d, msg, bytes(32))
s = Schnorr()
dF = BigUintFHE.new(d, ck)
ref = s.sign_with_k0(msg, k0, d)


def med(fn, n=7):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ctx.sync()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1e3


print("host cpus", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
print(f"encrypt 128 blocks (host)         {med(lambda: ck.encrypt_blocks(np.arange(128) % 4)):.2f} ms")
e = (1 << 255) + 12345
print(f"BigUintFHE.new 8 limbs (+upload)  {med(lambda: BigUintFHE.new(e, ck)):.2f} ms")
assert s.sign_fhe_with_k0(msg, k0, d, dF, ck, COMPAT) == ref
print(f"sign_fhe_with_k0 v0 compat        {med(lambda: s.sign_fhe_with_k0(msg, k0, d, dF, ck, COMPAT)):.2f} ms")
print(f"sign_with_k0 (plaintext)          {med(lambda: s.sign_with_k0(msg, k0, d)):.3f} ms")
