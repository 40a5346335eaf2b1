"""One op (compat / fast 256-bit mul, the 256-bit / encrypted division, or the 8-signature batch), run twice, the second time
timed; under rocprofv3 --kernel-trace its kernel timeline shows where the GPU waits for the host.
usage: rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/op_gaps.py compat|fast|div|divu32|batch8|sign
then:  python3 tools/op_gaps.py --analyze DIR/run_kernel_trace.csv"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if sys.argv[1] == "--analyze":
    import csv
    rows = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"]))
    # the timed run: kernels after the last gap longer than 50 ms (the untimed run's end, then the check)
    starts = [int(r["Start_Timestamp"]) for r in rows]
    ends = [int(r["End_Timestamp"]) for r in rows]
    cut = max(i for i in range(1, len(rows)) if starts[i] - ends[i - 1] > 50e6)
    rows, starts, ends = rows[cut:], starts[cut:], ends[cut:]
    busy, gaps = 0, []
    t_end = starts[0]
    for s, e in zip(starts, ends):
        if s > t_end:
            gaps.append(s - t_end)
        busy += max(0, e - max(s, t_end))
        t_end = max(t_end, e)
    span = t_end - starts[0]
    gaps.sort(reverse=True)
    print(f"kernels {len(rows)}, span {span / 1e6:.1f} ms, busy {busy / 1e6:.1f} ms, idle {sum(gaps) / 1e6:.1f} ms "
          f"in {len(gaps)} gaps; largest {[round(g / 1e6, 2) for g in gaps[:12]]} ms; "
          f"gaps > 0.1 ms: {sum(g for g in gaps if g > 1e5) / 1e6:.1f} ms")
    sys.exit(0)

import torch  # noqa: E402,F401  (one HIP runtime: torch's, loaded first)

sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
from fhe_sign import COMPAT, FAST, BigUintFHE, Context, FheUint256, generate_keys, set_server_key  # noqa: E402

op = sys.argv[1]
ck, sk = generate_keys(seed=0x5167)
ctx = Context(0)
ctx.set_server_key(sk)
set_server_key(ctx)
a, b = (1 << 255) - 12345, (1 << 254) + 777
if op in ("compat", "fast"):
    A, B = BigUintFHE.new(a, ck), BigUintFHE.new(b, ck)
    fn = lambda: A.mul(B, COMPAT if op == "compat" else FAST).to_biguint(ck)  # noqa: E731
elif op == "batch8":  # bench.py's config-5b batch: BIP-340 vectors 0, 1, 2, 15, 16, 17, 18, 0 as one schedule
    import csv
    from fhe_sign import Schnorr, compute_nonce
    rows = {r["index"]: r for r in csv.DictReader(open(os.path.join(ROOT, "tests", "golden", "bip340_vectors.csv")))}
    jobs = []
    for idx in ("0", "1", "2", "15", "16", "17", "18", "0"):
        dd = int(rows[idx]["secret key"], 16)
        mm, aux = bytes.fromhex(rows[idx]["message"]), bytes.fromhex(rows[idx]["aux_rand"])
        jobs.append((mm, compute_nonce(dd, mm, aux), dd, BigUintFHE.new(dd, ck)))
    fn = lambda: Schnorr().sign_fhe_with_k0_batch(jobs, ck, COMPAT)  # noqa: E731
elif op == "sign":  # sign_fhe_with_k0, BIP-340 vector 0 (fused column form)
    from fhe_sign import Schnorr, compute_nonce
    d0, msg0 = 3, bytes(32)
    k00 = compute_nonce(d0, msg0, bytes(32))
    dF0 = BigUintFHE.new(d0, ck)
    fn = lambda: Schnorr().sign_fhe_with_k0(msg0, k00, d0, dF0, ck, COMPAT)  # noqa: E731
elif op == "divu32":  # 256-bit / public u32 (the residue split)
    A = FheUint256.try_encrypt(a, ck)
    fn = lambda: (A // 0xC0FFEE01).decrypt(ck)  # noqa: E731
else:
    d = (1 << 127) | 12345
    A, D = FheUint256.try_encrypt(a, ck), FheUint256.try_encrypt(d, ck)
    fn = lambda: A.div_rem(D)[0].decrypt(ck)  # noqa: E731
fn()
ctx.sync()
time.sleep(0.2)
t0 = time.perf_counter()
fn()
ctx.sync()
print(f"{op}: {time.perf_counter() - t0:.3f} s", flush=True)
ctx.close()
