"""One process's timing of the classic throughput kernel of a library build (product or a
tools/build_variant.sh variant): HIP-event ms and clock-probe CU-cycles per PBS over `reps` launches
at B distinct encryptions.  usage: python3 tools/qy2_probe.py PKG_DIR KIND(4 qy, 5 qy2) [B] [reps] [mb: multi-bit keys]"""
import hashlib
import os
import sys

pkg = os.path.abspath(sys.argv[1])
sys.path.insert(0, pkg)
import numpy as np  # noqa: E402

import fhe_sign  # noqa: E402
from fhe_sign import Context, generate_keys, multi_bit_params  # noqa: E402

assert os.path.dirname(fhe_sign.__file__).startswith(pkg), fhe_sign.__file__
kind = int(sys.argv[2])
B = int(sys.argv[3]) if len(sys.argv) > 3 else 32768
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
ck, sk = generate_keys(multi_bit_params() if sys.argv[5:6] == ["mb"] else None, seed=1)
ctx = Context(0)
ctx.set_server_key(sk)
ctx.set_br_kernel(kind)
lid = ctx.lut([(m + 1) % 16 for m in range(16)])
cts = ck.encrypt_blocks(np.arange(B) % 16)
d_in, d_out, d_lut = ctx.alloc(cts.nbytes), ctx.alloc(cts.nbytes), ctx.alloc(B * 4)
ctx.h2d(d_in, cts)
ctx.h2d(d_lut, np.full(B, lid, np.uint32))
ctx.pbs_device(d_in, B, d_lut, d_out)
ctx.enable_timing(True)
ms, cyc, ghz_l = [], [], []
for _ in range(reps):
    ctx.enable_clock(True)
    ctx.pbs_device(d_in, B, d_lut, d_out)
    br = ctx.last_pbs_timing()[1]
    cy, tk, wg = ctx.read_clock()
    ctx.enable_clock(False)
    ghz = cy / tk * 0.1
    ms.append(br)
    ghz_l.append(ghz)
    cyc.append(br * 1e-3 * ghz * 1e9 * 256 / B)
o = np.zeros_like(cts)
ctx.d2h(o, d_out)
ok = all(ck.decrypt_block(o[i]) == (i % 16 + 1) % 16 for i in range(0, B, 97))
print(f"{os.path.basename(os.path.dirname(pkg)) or pkg} kind={kind} B={B}: {min(ms):.2f} ms (runs {' '.join(f'{x:.1f}' for x in ms)}), "
      f"{min(cyc) / 1e6:.4f} M CU-cycles/PBS, {max(ghz_l):.3f} GHz, decrypt_ok={ok}, "
      f"out_sha={hashlib.sha256(o.tobytes()).hexdigest()[:16]}", flush=True)
