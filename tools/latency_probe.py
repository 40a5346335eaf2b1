"""Blind-rotate kernel choice: batch-size sweep of the latency (wide) vs throughput (narrow) kernel."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
import numpy as np
from fhe_sign import Context, generate_keys
ck, sk = generate_keys(seed=1)
ctx = Context(0); ctx.set_server_key(sk)
lid = ctx.lut([(m + 1) % 16 for m in range(16)])
Bmax = 8192
cts = np.stack([ck.encrypt_block(m % 16) for m in range(64)])
cts = np.ascontiguousarray(np.concatenate([cts] * (Bmax // 64)))
d_in = ctx.alloc(cts.nbytes); d_out = ctx.alloc(cts.nbytes); d_lut = ctx.alloc(Bmax * 4)
ctx.h2d(d_in, cts); ctx.h2d(d_lut, np.full(Bmax, lid, np.uint32))
ctx.enable_timing(True)
for B in [1, 16, 64, 128, 256, 512, 768, 1024, 2048, 4096, 8192]:
    row = [B]
    for thr in (0, 1 << 30):
        ctx.set_wide_threshold(thr)
        ctx.pbs_device(d_in, B, d_lut, d_out); ctx.sync()
        best = 1e9
        for _ in range(2 if B >= 2048 else 3):
            ctx.pbs_device(d_in, B, d_lut, d_out)
            ks, br = ctx.last_pbs_timing()
            best = min(best, br)
        row += [round(ks, 3), round(best, 3)]
        out = np.zeros((B, 2049), np.uint64); ctx.d2h(out, d_out)
        assert all(ck.decrypt_block(out[i]) == ((i % 64) % 16 + 1) % 16 for i in range(0, B, max(1, B // 16)))
    print("B=%5d  narrow: ks %.3f br %.3f ms | wide: ks %.3f br %.3f ms  -> wide PBS/s %.0f narrow PBS/s %.0f" %
          (row[0], row[1], row[2], row[3], row[4], B / (row[4] + row[3]) * 1e3, B / (row[2] + row[1]) * 1e3), flush=True)
