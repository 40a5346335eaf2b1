"""Blind-rotate kernel choice: batch-size sweep of the latency kernel (wide, 8 waves/ciphertext) vs
the throughput kernel (quad: 4 waves), for the classic and the multi-bit (grouping 2) blind rotation.
Usage: latency_probe.py [classic|multibit ...] [--max B]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
import numpy as np
from fhe_sign import Context, default_params, generate_keys, multi_bit_params

argv = sys.argv[1:]
Bmax = 8192
if "--max" in argv:
    i = argv.index("--max")
    Bmax = int(argv[i + 1])
    del argv[i:i + 2]
args = argv
sizes = [b for b in [1, 16, 64, 128, 256, 320, 384, 512, 640, 768, 1024, 1536, 2048, 2304, 3072, 4096, 8192] if b <= Bmax]
for kind in (args or ["classic", "multibit"]):
    P = multi_bit_params() if kind == "multibit" else default_params()
    ck, sk = generate_keys(P, seed=1)
    ctx = Context(0); ctx.set_server_key(sk)
    lid = ctx.lut([(m + 1) % 16 for m in range(16)])
    cts = np.stack([ck.encrypt_block(m % 16) for m in range(64)])
    cts = np.ascontiguousarray(np.concatenate([cts] * (Bmax // 64 or 1))[:Bmax])
    d_in = ctx.alloc(cts.nbytes); d_out = ctx.alloc(cts.nbytes); d_lut = ctx.alloc(Bmax * 4)
    ctx.h2d(d_in, cts); ctx.h2d(d_lut, np.full(Bmax, lid, np.uint32))
    ctx.enable_timing(True)
    for B in sizes:
        res = {}
        for name, thr in (("wide", 1 << 30), ("quad", 0)):
            ctx.set_wide_threshold(thr)
            ctx.pbs_device(d_in, B, d_lut, d_out); ctx.sync()
            best = 1e9
            for _ in range(2 if B >= 2048 else 3):
                ctx.pbs_device(d_in, B, d_lut, d_out)
                ks, br = ctx.last_pbs_timing()
                best = min(best, br)
            res[name] = (ks, best)
            out = np.zeros((B, 2049), np.uint64); ctx.d2h(out, d_out)
            assert all(ck.decrypt_block(out[i]) == ((i % 64) % 16 + 1) % 16 for i in range(0, B, max(1, B // 16)))
        print("%-8s B=%5d  ks %.3f ms | br wide %.3f  quad %.3f ms" % (kind, B, res["quad"][0], res["wide"][1],
                                                                       res["quad"][1]), flush=True)
    ctx.close()
