"""Classic throughput kernels by level size: qy (one ciphertext per workgroup) against qy2 (two) at the
level sizes just above the latency kernel's threshold, where qy2 fills fewer workgroups, to choose the
size from which the engine uses qy2.  usage: python3 tools/qy2_sizes.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
import numpy as np  # noqa: E402

from fhe_sign import Context, generate_keys  # noqa: E402

ck, sk = generate_keys(seed=1)
ctx = Context(0)
ctx.set_server_key(sk)
ctx.set_wide_threshold(0)
lid = ctx.lut([(m + 1) % 16 for m in range(16)])
MAXB = 8192
cts = ck.encrypt_blocks(np.arange(MAXB) % 16)
d_in, d_out, d_lut = ctx.alloc(cts.nbytes), ctx.alloc(cts.nbytes), ctx.alloc(MAXB * 4)
ctx.h2d(d_in, cts)
ctx.h2d(d_lut, np.full(MAXB, lid, np.uint32))
ctx.enable_timing(True)
for B in (257, 320, 384, 512, 640, 768, 1024, 1280, 1536, 2048, 3072, 4096, 6144, 8192):
    best = {}
    for kind in (4, 5, 4, 5, 4, 5):
        ctx.set_br_kernel(kind)
        ctx.pbs_device(d_in, B, d_lut, d_out)
        t = ctx.last_pbs_timing()[1]
        best[kind] = min(best.get(kind, 1e9), t)
    print(f"B={B:5d}: qy {best[4]:7.3f} ms  qy2 {best[5]:7.3f} ms  qy2/qy {best[5] / best[4]:.3f}", flush=True)
