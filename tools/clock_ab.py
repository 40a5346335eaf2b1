"""Clock probe cost and readout (same process, interleaved): the classic throughput blind rotate at B
with fhe_ctx_enable_clock off / on, HIP-event kernel times of each, and the probe's shader clock and
CU-cycles per bootstrap.  usage: python3 tools/clock_ab.py [B] [rounds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
import numpy as np  # noqa: E402

from fhe_sign import Context, generate_keys  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
ck, sk = generate_keys(seed=1)
ctx = Context(0)
ctx.set_server_key(sk)
lid = ctx.lut([(m + 1) % 16 for m in range(16)])
cts = ck.encrypt_blocks(np.arange(B) % 16)
d_in, d_out, d_lut = ctx.alloc(cts.nbytes), ctx.alloc(cts.nbytes), ctx.alloc(B * 4)
ctx.h2d(d_in, cts)
ctx.h2d(d_lut, np.full(B, lid, np.uint32))
ctx.pbs_device(d_in, B, d_lut, d_out)
ctx.enable_timing(True)
t = {0: [], 1: []}
for rnd in range(rounds):
    for on in ((0, 1) if rnd % 2 == 0 else (1, 0)):
        ctx.enable_clock(bool(on))
        ctx.pbs_device(d_in, B, d_lut, d_out)
        br = ctx.last_pbs_timing()[1]
        t[on].append(br)
        if on:
            cy, tk, wg = ctx.read_clock()
            ghz = cy / tk * 0.1
            print(f"probe on: {br:.2f} ms, {ghz:.3f} GHz, {wg} workgroups, {cy / wg / 1e6:.3f} M cycles per workgroup, "
                  f"{br * 1e-3 * ghz * 1e9 * 256 / B / 1e6:.4f} M CU-cycles per PBS", flush=True)
        ctx.enable_clock(False)
o = np.zeros_like(cts)
ctx.d2h(o, d_out)
ok = all(ck.decrypt_block(o[i]) == (i % 16 + 1) % 16 for i in range(0, B, 97))
print(f"B={B}: probe off {min(t[0]):.2f} ms (runs {' '.join(f'{x:.1f}' for x in t[0])}), "
      f"on {min(t[1]):.2f} ms (runs {' '.join(f'{x:.1f}' for x in t[1])}) -> on/off {min(t[1]) / min(t[0]):.4f}; "
      f"decrypt_ok={ok}", flush=True)
sys.exit(0 if ok else 1)
