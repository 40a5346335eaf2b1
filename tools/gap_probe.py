"""GPU busy time vs wall time of the headline ops (compat 256-bit mul, sign_fhe_with_k0 v0):
run under rocprofv3 --kernel-trace, then tools/gap_probe.py --analyze DIR sums the kernel time
inside each op's window (marked by the probe's own timestamps) and the idle gaps between kernels.
usage (GPU box): rocprofv3 --kernel-trace -d gpurun_out/gap -o run --output-format csv -- python3 tools/gap_probe.py
                 python3 tools/gap_probe.py --analyze gpurun_out/gap"""
import csv, glob, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if sys.argv[1:2] == ["--analyze"]:
    d = sys.argv[2]
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f)))
    marks = json.load(open(os.path.join(d, "marks.json")))
    for name, t0, t1 in marks:
        # ops are separated by ctx.sync(): the op's kernels are those after the previous op's end
        sel = [k for k in ks if t0 <= k[0] <= t1]
        if not sel:
            print(name, "no kernels in window"); continue
        busy, last, gaps = 0, sel[0][0], []
        for s, e, n in sel:
            busy += e - max(s, last) if e > last else 0
            if s > last: gaps.append(s - last)
            last = max(last, e)
        span = sel[-1][1] - sel[0][0]
        big = sorted(gaps)[-5:]
        if os.environ.get("GAP_DETAIL"):  # where the gaps sit: (offset from t0, gap, kernel after it)
            last = sel[0][0]
            for s, e, n in sel:
                if s - last > 200_000:
                    print(f"   gap {(s - last) / 1e6:.2f} ms at +{(s - t0) / 1e6:.2f} ms before {n.split('(')[0][:40]}")
                last = max(last, e)
            print(f"   last kernel ends at +{(sel[-1][1] - t0) / 1e6:.2f} ms of {(t1 - t0) / 1e6:.2f}")
        print(f"{name}: wall {(t1 - t0) / 1e6:.1f} ms, first kernel at +{(sel[0][0] - t0) / 1e6:.1f} ms, kernel span "
              f"{span / 1e6:.1f} ms, busy {busy / 1e6:.1f} ms, idle gaps {sum(gaps) / 1e6:.1f} ms over {len(gaps)} "
              f"(largest {[round(g / 1e6, 2) for g in big]}), {len(sel)} kernels")
    sys.exit(0)
sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
import random
from fhe_sign import *
ck, sk = generate_keys(seed=9)
ctx = Context(0); ctx.set_server_key(sk); set_server_key(ctx)
rng = random.Random(0xF11E51)
a, b = rng.getrandbits(256) | 1 << 255, rng.getrandbits(256) | 1 << 255
A, B = BigUintFHE.new(a, ck), BigUintFHE.new(b, ck)
A.add(B, FAST); ctx.sync()
marks = []
def mark(name, fn):
    ctx.sync()
    t0 = time.clock_gettime_ns(time.CLOCK_BOOTTIME)
    r = fn(); ctx.sync()  # r held across the sync: the engine drops bootstraps nothing can read
    t1 = time.clock_gettime_ns(time.CLOCK_BOOTTIME)
    del r
    marks.append((name, t0, t1))
    print(name, (t1 - t0) / 1e6, "ms", flush=True)
for _ in range(2):
    mark("mul_compat", lambda: A.mul(B, COMPAT))
d = 3; msg = bytes(32); k0 = compute_nonce(d, msg, bytes(32)); dF = BigUintFHE.new(d, ck)
for _ in range(2):
    mark("sign", lambda: Schnorr().sign_fhe_with_k0(msg, k0, d, dF, ck, COMPAT))
out = os.environ.get("GAP_OUT", os.path.join(ROOT, "gpurun_out", "gap"))
os.makedirs(out, exist_ok=True)
json.dump(marks, open(os.path.join(out, "marks.json"), "w"))
