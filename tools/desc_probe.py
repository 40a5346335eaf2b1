"""One radix level through the engine's descriptor path: x & 0x55..55 on a 4096-bit radix (2048
univariate PBS in one KS + BR launch).  usage: python3 tools/desc_probe.py [package_dir] [bits]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.abspath(sys.argv[1]) if len(sys.argv) > 1 else os.path.join(ROOT, "fhe-sign_amd")
sys.path.insert(0, PKG)
import random
from fhe_sign import Context, FheUint, generate_keys, set_server_key, stats
bits = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
ck, sk = generate_keys(seed=3)
ctx = Context(0); ctx.set_server_key(sk); set_server_key(ctx)
rng = random.Random(1)
v = rng.getrandbits(bits)
X = FheUint.try_encrypt(v, ck, bits=bits)
mask = int("01" * (bits // 2), 2)
r = X & mask; ctx.sync()
ts = []
for _ in range(3):
    p0, l0 = stats(ctx); t0 = time.perf_counter(); r = X & mask; ctx.sync(); ts.append(time.perf_counter() - t0)
    p1, l1 = stats(ctx)
assert r.decrypt(ck) == v & mask
print(f"{os.path.basename(PKG)}: {bits}-bit & mask: {p1 - p0} PBS in {l1 - l0} level(s), best {min(ts) * 1e3:.1f} ms", flush=True)
