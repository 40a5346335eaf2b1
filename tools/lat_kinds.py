"""Latency-level blind rotate by kernel: the 8-wave latency kernel (wide) against the 4-wave throughput
kernels (quad, qx, qy) forced onto small batches (wide threshold 0), at B = 1 .. 512 distinct
encryptions, best of R launches each, every output checked by decryption.
usage: python3 tools/lat_kinds.py [--pkg DIR] [--kinds a,b] [R] [B ...]   (DIR: a tools/build_variant.sh build)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
argv = sys.argv[1:]
PKG, SEL = os.path.join(ROOT, "fhe-sign_amd"), None
while argv and argv[0].startswith("--"):
    if argv[0] == "--pkg":
        PKG = os.path.abspath(argv[1])
    elif argv[0] == "--kinds":
        SEL = argv[1].split(",")
    argv = argv[2:]
sys.path.insert(0, PKG)
import numpy as np  # noqa: E402

import fhe_sign  # noqa: E402
from fhe_sign import Context, generate_keys  # noqa: E402

assert os.path.dirname(fhe_sign.__file__).startswith(PKG), fhe_sign.__file__
R = int(argv[0]) if argv else 5
sizes = [int(b) for b in argv[1:]] or [1, 64, 256, 512]
KINDS = [k for k in (("wide", None), ("quad", 1), ("qx", 3), ("qy", 4)) if SEL is None or k[0] in SEL]
ck, sk = generate_keys(seed=1)
ctx = Context(0)
ctx.set_server_key(sk)
lid = ctx.lut([(m + 1) % 16 for m in range(16)])
Bmax = max(sizes)
cts = ck.encrypt_blocks(np.arange(Bmax) % 16)
d_in, d_out, d_lut = ctx.alloc(cts.nbytes), ctx.alloc(cts.nbytes), ctx.alloc(Bmax * 4)
ctx.h2d(d_in, cts)
ctx.h2d(d_lut, np.full(Bmax, lid, np.uint32))
ctx.enable_timing(True)
for B in sizes:
    res = {}
    for name, kind in KINDS:
        if kind is None:
            ctx.set_wide_threshold(1 << 30)
        else:
            ctx.set_wide_threshold(0)
            ctx.set_br_kernel(kind)
        ts = []
        for _ in range(R + 1):
            ctx.pbs_device(d_in, B, d_lut, d_out)
            ts.append(ctx.last_pbs_timing()[1])
        o = np.zeros((B, 2049), np.uint64)
        ctx.d2h(o, d_out)
        assert all(ck.decrypt_block(o[i]) == (i % 16 + 1) % 16 for i in range(B)), (name, B)
        res[name] = min(ts[1:])
    print(f"{os.path.basename(PKG)} B={B:4d}  " + "  ".join(f"{k} {v:.3f} ms" for k, v in res.items()), flush=True)
ctx.set_wide_threshold(256)
ctx.close()
