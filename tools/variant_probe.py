"""Throughput of one kernel variant built by tools/build_variant.sh (package dir given explicitly).
usage: python3 tools/variant_probe.py build_variants/NAME [B] [reps]"""
import os, sys, time
pkg = os.path.abspath(sys.argv[1])
sys.path.insert(0, pkg)
import numpy as np
import fhe_sign
assert os.path.dirname(fhe_sign.__file__).startswith(pkg), fhe_sign.__file__
from fhe_sign import Context, generate_keys
MB = os.environ.get("FHE_PROBE_MB") == "1"  # multi-bit (grouping 2) keys
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
distinct = len(sys.argv) > 4 and sys.argv[4] == "distinct"  # B independent encryptions, not 64 repeated
ck, sk = generate_keys(fhe_sign.multi_bit_params() if MB else None, seed=1)
ctx = Context(0); ctx.set_server_key(sk)
lid = ctx.lut([(m + 1) % 16 for m in range(16)])
if distinct:
    cts = np.ascontiguousarray(np.stack([ck.encrypt_block(m % 16) for m in range(B)]))
else:
    cts = np.stack([ck.encrypt_block(m % 16) for m in range(64)])
    cts = np.ascontiguousarray(np.concatenate([cts] * max(1, B // 64))[:B])
d_in = ctx.alloc(cts.nbytes); d_out = ctx.alloc(cts.nbytes); d_lut = ctx.alloc(B * 4)
ctx.h2d(d_in, cts); ctx.h2d(d_lut, np.full(B, lid, np.uint32))
ctx.enable_timing(True)
times = []
for r in range(reps):
    ctx.pbs_device(d_in, B, d_lut, d_out); ctx.sync()
    times.append(ctx.last_pbs_timing()[1])
best = min(times)
if reps > 3:
    print("per-rep br ms:", " ".join(f"{t:.1f}" for t in times), flush=True)
out = np.zeros_like(cts); ctx.d2h(out, d_out)
ok = all(ck.decrypt_block(out[i]) == ((i if distinct else i % 64) % 16 + 1) % 16 for i in range(0, B, 131))
print(f"{os.path.basename(pkg)}{' distinct' if distinct else ''}{' MB' if MB else ''}: B={B} br best {best:.2f} ms -> {B / best * 1e3:.0f} BR/s  decrypt_ok={ok}", flush=True)
