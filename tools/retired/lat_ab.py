"""RETIRED with tools/retired/br_wx_r4.hip (needs its build).  Same-box A/B of the classic latency blind-rotate kernels: br_wx.hip (1) against br_wide.hip (0),
interleaved, at level sizes 1, 64, 128, 256 (one ciphertext per CU); outputs compared word for word.
usage: python3 tools/lat_ab.py [rounds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
import numpy as np  # noqa: E402

from fhe_sign import Context, generate_keys  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
ck, sk = generate_keys(seed=1)
ctx = Context(0)
ctx.set_server_key(sk)
ctx.set_wide_threshold(1 << 30)
lid = ctx.lut([(m + 1) % 16 for m in range(16)])
B = 256
cts = ck.encrypt_blocks(np.arange(B) % 16)
d_in, d_out, d_lut = ctx.alloc(cts.nbytes), ctx.alloc(cts.nbytes), ctx.alloc(B * 4)
ctx.h2d(d_in, cts)
ctx.h2d(d_lut, np.full(B, lid, np.uint32))
ctx.enable_timing(True)
bad = False
for n in (1, 64, 128, 256):
    times, outs = {0: [], 1: []}, {}
    for rnd in range(rounds):
        for kind in (1, 0) if rnd % 2 == 0 else (0, 1):
            ctx.set_latency_kernel(kind)
            ctx.pbs_device(d_in, n, d_lut, d_out)
            times[kind].append(ctx.last_pbs_timing()[1])
            if kind not in outs:
                o = np.zeros((n, 2049), np.uint64)
                ctx.d2h(o, d_out)
                outs[kind] = o
    same = np.array_equal(outs[0], outs[1])
    ok = all(ck.decrypt_block(outs[1][i]) == (i % 16 + 1) % 16 for i in range(n))
    bad |= not (same and ok)
    w, x = min(times[0]), min(times[1])
    print(f"B={n}: wide {w:.3f} ms, wx {x:.3f} ms -> wx/wide {x / w:.3f} (wide runs "
          f"{' '.join(f'{t:.3f}' for t in times[0])}; wx runs {' '.join(f'{t:.3f}' for t in times[1])}) "
          f"identical={same} decrypt_ok={ok}", flush=True)
sys.exit(1 if bad else 0)
