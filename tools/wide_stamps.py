"""Per-CMUX critical path of the latency blind rotate (br_wide.hip, classic) from the WIDE_STAMPS
variant build: lane 0 of every wave records s_memtime at the phase boundaries of 32 CMUX
iterations.  usage (GPU box): python3 tools/wide_stamps.py [B ...]   (build: tools/wide_stamps.sh)
Phases (stamp k -> k+1; factored CMUX, round 3): 0 top -> 1 digits (with the deferred reduction),
monomial DMA, key loads issued, monomial factor -> (2, 3 empty) -> 4 forward A..D + cross store ->
5 barrier X -> 6 phase E (each point and polynomial once, paired swaps) + MAC + (X^a - 1) -> 7 inverse first stage + store ->
8 barrier Y -> 9 inverse D..A + accumulate."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VAR = os.path.join(ROOT, "build_variants", os.environ.get("WS_VARIANT", "wide_stamps"))
sys.path.insert(0, VAR)
import numpy as np  # noqa: E402
from fhe_sign import Context, generate_keys, load  # noqa: E402

NAMES = ["digits+loads+e", "-", "-", "fwd A..D+store", "barrier X", "E + MAC + (X^a-1)",
         "inv first+store", "barrier Y", "inv D..A+acc", "loop tail"]
WS_CT, WS_IT, WS_N = 2, 32, 10

lib = load()
assert lib._name.startswith(VAR), lib._name
fn = lib.fhe_debug_wide_stamps
fn.restype = C.c_int
fn.argtypes = [C.POINTER(C.c_uint64), C.c_size_t]

ck, sk = generate_keys(seed=1)
ctx = Context(0)
ctx.set_server_key(sk)
ctx.set_wide_threshold(1 << 30)
lid = ctx.lut([(m + 1) % 16 for m in range(16)])
sizes = [int(b) for b in sys.argv[1:]] or [1, 256]
Bmax = max(sizes)
cts = np.ascontiguousarray(np.stack([ck.encrypt_block(m % 16) for m in range(Bmax)]))
d_in, d_out, d_lut = ctx.alloc(cts.nbytes), ctx.alloc(cts.nbytes), ctx.alloc(Bmax * 4)
ctx.h2d(d_in, cts)
ctx.h2d(d_lut, np.full(Bmax, lid, np.uint32))
ctx.enable_timing(True)
for B in sizes:
    ms = []
    for _ in range(3):
        ctx.pbs_device(d_in, B, d_lut, d_out)
        ms.append(ctx.last_pbs_timing()[1])
    ctx.sync()
    buf = np.zeros(WS_CT * 8 * WS_IT * WS_N, np.uint64)
    assert fn(buf.ctypes.data_as(C.POINTER(C.c_uint64)), buf.size) == 0
    st = buf.reshape(WS_CT, 8, WS_IT, WS_N).astype(np.int64)
    s0 = st[0]  # ciphertext 0: [wave][iteration][stamp]
    valid = (s0 != 0).all(axis=2).all(axis=0)  # iterations every wave stamped (a = 0 skips leave zeros)
    it = np.nonzero(valid)[0]
    per_iter = np.diff(s0[0, it, 0])
    per_iter = per_iter[np.diff(it) == 1]
    print(f"B={B}: BR {min(ms):.3f} ms -> {min(ms) * 1e3 / 834:.3f} us per CMUX; stamped iterations {len(it)}; "
          f"clock ticks per CMUX (wave 0, consecutive): median {np.median(per_iter):.0f}")
    # phase durations per wave: stamp k+1 - stamp k; the last phase to the next iteration's top
    rows = []
    for k in range(WS_N - 1):
        d = s0[:, it, k + 1] - s0[:, it, k]
        rows.append((NAMES[k], np.median(d, axis=1)))
    tail = s0[:, it[1:], 0] - s0[:, it[:-1], 9]
    tail = tail[:, np.diff(it) == 1]
    rows.append((NAMES[9], np.median(tail, axis=1) if tail.size else np.zeros(8)))
    print("  phase               " + " ".join(f"w{w:<5d}" for w in range(8)) + "  max   share")
    tot = sum(r[1].max() for r in rows)
    for name, d in rows:
        print(f"  {name:<19s} " + " ".join(f"{v:6.0f}" for v in d) + f" {d.max():6.0f} {d.max() / tot:5.1%}")
    # barrier skew: when each wave arrives at / leaves the barriers (relative to the earliest)
    for k, lab in ((4, "arrive X"), (7, "arrive Y")):
        arr = s0[:, it, k] - s0[:, it, k].min(axis=0)
        print(f"  {lab}: median lag per wave " + " ".join(f"{v:5.0f}" for v in np.median(arr, axis=1)))
    sys.stdout.flush()
ctx.close()
