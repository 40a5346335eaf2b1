"""Same-box A/B of the classic throughput kernels k_blind_rotate_qy (FHE_BR_QY, one ciphertext per
workgroup) and k_blind_rotate_qy2 (FHE_BR_QY2, two per workgroup sharing the key stream), interleaved,
on B distinct encryptions resident on the device; every output word compared; the clock probe gives
each launch's shader clock, so the comparison is also reported in CU-cycles per bootstrap.
usage: python3 tools/qy2_ab.py [B] [rounds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
import numpy as np  # noqa: E402

from fhe_sign import Context, generate_keys  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
QY, QY2, QY4 = 4, 5, 6
KINDS = (QY, QY2, QY4)
NAME = {QY: "qy", QY2: "qy2", QY4: "qy4"}
ck, sk = generate_keys(seed=1)
ctx = Context(0)
ctx.set_server_key(sk)
lid = ctx.lut([(m + 1) % 16 for m in range(16)])
cts = ck.encrypt_blocks(np.arange(B) % 16)
d_in, d_out, d_lut = ctx.alloc(cts.nbytes), ctx.alloc(cts.nbytes), ctx.alloc(B * 4)
ctx.h2d(d_in, cts)
ctx.h2d(d_lut, np.full(B, lid, np.uint32))
for kind in KINDS:  # warm-up
    ctx.set_br_kernel(kind)
    ctx.pbs_device(d_in, B, d_lut, d_out)
ctx.enable_timing(True)
outs, times, cyc = {}, {k: [] for k in KINDS}, {k: [] for k in KINDS}
for rnd in range(rounds):
    for kind in KINDS if rnd % 2 == 0 else KINDS[::-1]:
        ctx.set_br_kernel(kind)
        ctx.enable_clock(True)
        ctx.pbs_device(d_in, B, d_lut, d_out)
        br = ctx.last_pbs_timing()[1]
        cy, tk, wg = ctx.read_clock()
        ctx.enable_clock(False)
        ghz = cy / tk * 0.1
        times[kind].append(br)
        cyc[kind].append(br * 1e-3 * ghz * 1e9 * 256 / B)
        if kind not in outs:
            o = np.zeros_like(cts)
            ctx.d2h(o, d_out)
            outs[kind] = o
same = all(np.array_equal(outs[QY], outs[k]) for k in KINDS)
ok = all(ck.decrypt_block(outs[QY4][i]) == (i % 16 + 1) % 16 for i in range(0, B, 97))
base = min(times[QY])
print(f"B={B}: " + "; ".join(f"{NAME[k]} {min(times[k]):.2f} ms (runs {' '.join(f'{t:.1f}' for t in times[k])}; "
                             f"{min(cyc[k]) / 1e6:.4f} M CU-cycles/PBS; x{min(times[k]) / base:.3f})" for k in KINDS)
      + f"; identical={same} decrypt_ok={ok}", flush=True)
sys.exit(0 if same and ok else 1)
