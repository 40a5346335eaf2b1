"""Same-box A/B of two classic throughput blind-rotate kernels (default: br_qx.hip, FHE_BR_QX = 3,
against br_quad.hip, FHE_BR_QUAD = 1; br_qy.hip is 4), interleaved, on one batch of B distinct
encryptions resident on the device; every output word of the two kernels compared.
usage: python3 tools/br_ab.py [B] [rounds] [kind_a kind_b]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
import numpy as np  # noqa: E402

from fhe_sign import Context, generate_keys  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
KA, KB = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (3, 1)
NAME = {1: "quad", 3: "qx", 4: "qy"}
ck, sk = generate_keys(seed=1)
ctx = Context(0)
ctx.set_server_key(sk)
lid = ctx.lut([(m + 1) % 16 for m in range(16)])
cts = ck.encrypt_blocks(np.arange(B) % 16)
d_in, d_out, d_lut = ctx.alloc(cts.nbytes), ctx.alloc(cts.nbytes), ctx.alloc(B * 4)
ctx.h2d(d_in, cts)
ctx.h2d(d_lut, np.full(B, lid, np.uint32))
ctx.enable_timing(True)
outs, times = {}, {KA: [], KB: []}
for rnd in range(rounds):
    for kind in (KA, KB) if rnd % 2 == 0 else (KB, KA):
        ctx.set_br_kernel(kind)
        ctx.pbs_device(d_in, B, d_lut, d_out)
        times[kind].append(ctx.last_pbs_timing()[1])
        if kind not in outs:
            o = np.zeros_like(cts)
            ctx.d2h(o, d_out)
            outs[kind] = o
same = np.array_equal(outs[KA], outs[KB])
ok = all(ck.decrypt_block(outs[KA][i]) == (i % 16 + 1) % 16 for i in range(0, B, 97))
q, x = min(times[KB]), min(times[KA])
na, nb = NAME[KA], NAME[KB]
print(f"B={B}: {nb} {q:.2f} ms (runs {' '.join(f'{t:.1f}' for t in times[KB])}), "
      f"{na} {x:.2f} ms (runs {' '.join(f'{t:.1f}' for t in times[KA])}) -> {na}/{nb} {x / q:.3f}; "
      f"identical={same} decrypt_ok={ok}", flush=True)
if not (same and ok):
    sys.exit(1)
