"""Same-process A/B of the encrypted 256-bit division's leading radix-16 width (FHE_DIV_R16, read per
call): quotient + remainder of a random 256-bit value by a 128-bit-valued divisor, both encrypted, each
setting timed in interleaved rounds (median), every result checked.
usage (GPU box): python3 tools/div_ab.py [lead ...]   (default 0 16 32 48); FHE_PROBE_MB=1: multi-bit keys"""
import os
import random
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
from fhe_sign import Context, FheUint256, generate_keys, multi_bit_params, set_server_key  # noqa: E402

leads = [int(x) for x in sys.argv[1:]] or [0, 16, 32, 48]
ck, sk = generate_keys(multi_bit_params() if os.environ.get("FHE_PROBE_MB") == "1" else None, seed=7)
ctx = Context(0)
ctx.set_server_key(sk)
set_server_key(ctx)
rng = random.Random(3)
a, d = rng.getrandbits(256), rng.getrandbits(128) | 1 << 127
A, D = FheUint256.try_encrypt(a, ck), FheUint256.try_encrypt(d, ck)
times = {L: [] for L in leads}
for rnd in range(3):
    for L in leads:
        os.environ["FHE_DIV_R16"] = str(L)
        ctx.sync()
        t0 = time.perf_counter()
        q, r = A.div_rem(D)
        ctx.sync()
        dt = time.perf_counter() - t0
        assert (q.decrypt(ck), r.decrypt(ck)) == (a // d, a % d), L
        times[L].append(dt)
        print(f"round {rnd} lead {L:3d}: {dt:.4f} s", flush=True)
for L in leads:
    print(f"lead {L:3d}: median {statistics.median(times[L]):.4f} s  min {min(times[L]):.4f} s")
