"""Per-level schedule trace of the headline ops (FHE_TRACE_LEVELS=1: the engine synchronizes after
every level and prints its PBS count and wall time to stderr).
usage: FHE_TRACE_LEVELS=1 [FHE_PROBE_MB=1] python3 tools/level_trace.py [op ...]  (ops: mul_compat mul_fast sign div_enc)"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import random
from fhe_sign import *

MB = os.environ.get("FHE_PROBE_MB") == "1"  # multi-bit (grouping 2) keys
ck, sk = generate_keys(multi_bit_params() if MB else None, seed=9)
ctx = Context(0); ctx.set_server_key(sk); set_server_key(ctx)
rng = random.Random(0xF11E51)
a, b = rng.getrandbits(256) | 1 << 255, rng.getrandbits(256) | 1 << 255
A, B = BigUintFHE.new(a, ck), BigUintFHE.new(b, ck)
A.add(B, FAST); ctx.sync()
ops = sys.argv[1:] or ["mul_compat", "mul_fast", "sign"]
for op in ops:
    print(f"== {op}", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    if op == "mul_compat": A.mul(B, COMPAT)
    elif op == "mul_fast": A.mul(B, FAST)
    elif op == "sign":
        d = 3; msg = bytes(32); k0 = compute_nonce(d, msg, bytes(32)); dF = BigUintFHE.new(d, ck)
        Schnorr().sign_fhe_with_k0(msg, k0, d, dF, ck, COMPAT)
    elif op == "sign_batch8":
        import csv
        rows = {r["index"]: r for r in csv.DictReader(open(os.path.join(ROOT, "tests", "golden", "bip340_vectors.csv")))}
        jobs = []
        for idx in ("0", "1", "2", "15", "16", "17", "18", "0"):
            dd = int(rows[idx]["secret key"], 16)
            mm, aux = bytes.fromhex(rows[idx]["message"]), bytes.fromhex(rows[idx]["aux_rand"])
            jobs.append((mm, compute_nonce(dd, mm, aux), dd, BigUintFHE.new(dd, ck)))
        t0 = time.perf_counter()
        Schnorr().sign_fhe_with_k0_batch(jobs, ck, COMPAT)
    elif op == "div_enc":
        FheUint64.try_encrypt(a % 2**64, ck).div_rem(FheUint64.try_encrypt(b % 2**40, ck))
    print(f"== {op} host graph built {time.perf_counter() - t0:.4f} s", file=sys.stderr, flush=True)
    ctx.sync()
    print(f"== {op} total {time.perf_counter() - t0:.4f} s", file=sys.stderr, flush=True)
