"""Same-process A/B of the division by a PUBLIC divisor: the multiplier method against the residue split
(FHE_SCALAR_DIV_RESIDUE=0 / 1, read per call), 256-bit dividend by 5, a u32 and a u64 (the bench's
div256_by_5 / div256_by_u32 shapes) and the 128-bit one by a u32, plus the remainder by a u32; 5
interleaved rounds, medians, every result checked.
usage (GPU box): python3 tools/scalar_div_ab.py"""
import os
import random
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
from fhe_sign import Context, FheUint128, FheUint256, generate_keys, set_server_key  # noqa: E402

ck, sk = generate_keys(seed=7)
ctx = Context(0)
ctx.set_server_key(sk)
set_server_key(ctx)
rng = random.Random(5)
a, a128 = rng.getrandbits(256), rng.getrandbits(128)
du32, du64 = rng.getrandbits(32) | 1 << 31, rng.getrandbits(64) | 1 << 63
A, A128 = FheUint256.try_encrypt(a, ck), FheUint128.try_encrypt(a128, ck)
legs = [("256/5", lambda: A // 5, a // 5), ("256/u32", lambda: A // du32, a // du32),
        ("256/u64", lambda: A // du64, a // du64), ("128/u32", lambda: A128 // du32, a128 // du32),
        ("256%u32", lambda: A % du32, a % du32)]
modes = ["0", "1"]
times = {(n, m): [] for n, _, _ in legs for m in modes}
for rnd in range(5):
    for name, fn, want in legs:
        for m in modes:
            os.environ["FHE_SCALAR_DIV_RESIDUE"] = m
            ctx.sync()
            t0 = time.perf_counter()
            r = fn()
            ctx.sync()
            dt = time.perf_counter() - t0
            assert r.decrypt(ck) == want, (name, m)
            times[(name, m)].append(dt)
    print(f"round {rnd} done", flush=True)
for name, _, _ in legs:
    med = {m: statistics.median(times[(name, m)]) for m in modes}
    print(f"{name:8s} multiplier {med['0'] * 1e3:7.1f} ms   residue {med['1'] * 1e3:7.1f} ms   "
          f"({(med['1'] / med['0'] - 1) * 100:+.1f} %)")
