"""Quick PBS throughput probe (device-resident batch), used while developing kernels."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("FHE_PROBE_PKG") or os.path.join(ROOT, "fhe-sign_amd"))  # a build_variants/ dir
import numpy as np
import fhe_sign
from fhe_sign import Context, generate_keys
MB = os.environ.get("FHE_PROBE_MB") == "1"  # multi-bit (grouping 2) keys

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
t0 = time.time()
ck, sk = generate_keys(fhe_sign.multi_bit_params() if MB else None, seed=1)
print(f"keygen {time.time()-t0:.2f}s", flush=True)
ctx = Context(0)
t0 = time.time(); ctx.set_server_key(sk); print(f"set_server_key {time.time()-t0:.2f}s", flush=True)
if os.environ.get("FHE_PROBE_BR"):  # throughput kernel: 4 = br_qy (classic default), 3 = br_qx, 1 = br_quad
    ctx.set_br_kernel(int(os.environ["FHE_PROBE_BR"]))
lid = ctx.lut([(m + 1) % 16 for m in range(16)])
cts = np.stack([ck.encrypt_block(m % 16) for m in range(64)])
cts = np.ascontiguousarray(np.concatenate([cts] * max(1, -(-B // 64)))[:B])
d_in = ctx.alloc(cts.nbytes); d_out = ctx.alloc(cts.nbytes); d_lut = ctx.alloc(B * 4)
ctx.h2d(d_in, cts); ctx.h2d(d_lut, np.full(B, lid, np.uint32))
ctx.enable_timing(True)
for r in range(reps):
    t0 = time.time()
    ctx.pbs_device(d_in, B, d_lut, d_out)
    ctx.sync()
    dt = time.time() - t0
    ks, br = ctx.last_pbs_timing()
    print(f"B={B} wall {dt*1e3:.1f} ms  ks {ks:.2f} ms  br {br:.2f} ms  -> {B/dt:.0f} PBS/s", flush=True)
out = np.zeros_like(cts); ctx.d2h(out, d_out)
print("decrypt check", all(ck.decrypt_block(out[i]) == (i % 64 % 16 + 1) % 16 for i in range(0, B, 131)))
