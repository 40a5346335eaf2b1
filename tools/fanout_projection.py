"""Config 5 (one op fanned over N GPUs) projected from one GPU: the engine runs the op with N emulated
ranks at the production split (levels of >= 257 bootstraps split, fhe_ctx_set_fanout), the level log
records every level's size and whether it was split, and rank 0's share of each level is then
REPLAYED on this GPU as raw bootstrap launches (keyswitch + blind rotate of that many ciphertexts,
each level synchronised), which is what one rank of a real N-GPU run computes.  The all-gathers' own
cost, per split level (G bootstrap outputs of 16,392 B): allgather_copy_s = a measured device copy of
the level's whole gather buffer on this GPU (the bytes every rank writes into its gather buffer, the
scatter's read included as a second copy), allgather_link_s = the (W - 1) / W of it each rank receives
at XGMI_GBS (one 153 GB/s xGMI link: the conservative ring bound) plus COLL_LAT_S per collective.
projected_rank_s = rank_replay_s + allgather_copy_s + allgather_link_s + host_call_s (the host graph
build runs on every rank; for the signer, which decrypts inside the call, host_call_s is its wall time
minus its levels replayed at one rank).  emulated_wall_s is NOT a projection: one GPU computing every rank's slice
(it grows with the rank count).
usage: python3 tools/fanout_projection.py [ranks...]   (default 1 2 4 8)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401 -- before the engine: one HIP runtime in the process (tools/torch_hip_probe.py)

from fhe_sign import (COMPAT, FAST, LEVEL_SPLIT, BigUintFHE, Context, Schnorr, compute_nonce,  # noqa: E402
                      generate_keys, level_log, rank_pbs, set_server_key)

ranks_list = [int(x) for x in sys.argv[1:]] or [1, 2, 4, 8]
g = json.load(open(os.path.join(ROOT, "tests", "golden", "biguint_vectors.json")))["mul"][0]
val = lambda limbs: sum(int(x) << (32 * i) for i, x in enumerate(limbs))  # noqa: E731
a, b = val(g["a"]), val(g["b"])
ck, sk = generate_keys(seed=0xFA11)
ctx = Context(0)
ctx.set_server_key(sk)
set_server_key(ctx)
lid = ctx.lut([(m + 1) % 16 for m in range(16)])
MAXB = 32768
cts = ck.encrypt_blocks(np.arange(MAXB) % 16)
d_in, d_out, d_lut = ctx.alloc(cts.nbytes), ctx.alloc(cts.nbytes), ctx.alloc(MAXB * 4)
ctx.h2d(d_in, cts)
ctx.h2d(d_lut, np.full(MAXB, lid, np.uint32))


XGMI_GBS = 153.0    # one xGMI link, GB/s (MI355X: 7 links per GPU)
COLL_LAT_S = 30e-6  # per RCCL collective (launch + ring latency, order of magnitude)


def copy_time(level_bytes):
    """measured: each split level's gather buffer copied device to device twice (the rank segments
    landing in it, and the scatter into the block slots), levels synchronised"""
    import torch
    if not level_bytes:
        return 0.0
    m = max(level_bytes)
    src = torch.empty(m, dtype=torch.uint8, device="cuda")
    dst = torch.empty(m, dtype=torch.uint8, device="cuda")
    dst.copy_(src)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for nb in level_bytes:
        dst[:nb].copy_(src[:nb])
        src[:nb].copy_(dst[:nb])
        torch.cuda.synchronize()
    return time.perf_counter() - t0


def replay(sizes):
    """wall time of launching these level sizes back to back, each level synchronised"""
    ctx.pbs_device(d_in, 256, d_lut, d_out)
    ctx.sync()
    t0 = time.perf_counter()
    for k in sizes:
        if k:
            ctx.pbs_device(d_in, min(k, MAXB), d_lut, d_out)
            ctx.sync()
    return time.perf_counter() - t0


A, B = BigUintFHE.new(a, ck), BigUintFHE.new(b, ck)
d, msg = 3, bytes(32)
k0 = compute_nonce(d, msg, bytes(32))
dF = BigUintFHE.new(d, ck)
s = Schnorr()
ops = {
    "biguint256_mul_compat": lambda: A.mul(B, COMPAT),
    "biguint256_mul_fast": lambda: A.mul(B, FAST),
    "sign_fhe_with_k0_v0_compat": lambda: s.sign_fhe_with_k0(msg, k0, d, dF, ck, COMPAT),
}
ref = {"biguint256_mul_compat": [int(x) for x in g["out"]], "biguint256_mul_fast": a * b,
       "sign_fhe_with_k0_v0_compat": s.sign_with_k0(msg, k0, d)}
rows = []
host_only = {}
for W in ranks_list:
    ctx.set_fanout(min_level=257, emulate_ranks=W if W > 1 else 0)
    for name, fn in ops.items():
        fn()  # warm-up (pools, LUTs)
        ctx.sync()
        level_log(ctx)
        p0 = rank_pbs(ctx)
        t0 = time.perf_counter()
        r = fn() if name.startswith("sign") else fn()
        t_call = time.perf_counter() - t0  # sign: includes its own host reads; mul: the graph build
        ctx.sync()
        t_op = time.perf_counter() - t0
        log = level_log(ctx)
        p1 = rank_pbs(ctx)
        if name == "biguint256_mul_compat":
            assert r.decrypt_limbs(ck) == ref[name]
        elif name == "biguint256_mul_fast":
            assert r.to_biguint(ck) == ref[name]
        else:
            assert r == ref[name]
        share = []
        for e in log:
            G, split = e & ~LEVEL_SPLIT, bool(e & LEVEL_SPLIT)
            share.append((G + W - 1) // W if split else G)
        t_rank = replay(share)
        if name.startswith("sign"):
            # the signer reads its result on the host (decryption), so t_call holds the GPU levels too:
            # its host-only part is the call's wall time minus its levels replayed, taken at one rank
            # (the host work does not depend on the rank count; emulated ranks would inflate it)
            if W == 1 or name not in host_only:
                host_only[name] = max(0.0, t_op - t_rank) if W == 1 else t_call
            t_call = host_only[name]
        split_pbs = sum(e & ~LEVEL_SPLIT for e in log if e & LEVEL_SPLIT)
        nsplit = sum(1 for e in log if e & LEVEL_SPLIT)
        level_bytes = [(e & ~LEVEL_SPLIT) * 2049 * 8 for e in log if e & LEVEL_SPLIT]
        t_copy = copy_time(level_bytes) if W > 1 else 0.0
        t_link = (sum(level_bytes) * (W - 1) / W / (XGMI_GBS * 1e9) + nsplit * COLL_LAT_S) if W > 1 else 0.0
        row = {"op": name, "ranks": W, "levels": len(log), "split_levels": nsplit,
               "pbs": sum(e & ~LEVEL_SPLIT for e in log), "rank_pbs": p1 - p0,
               "redundant_levels": sum(1 for e in log if not e & LEVEL_SPLIT),
               "allgather_mb": round(split_pbs * 2049 * 8 / 1e6, 1),
               "rank_replay_s": round(t_rank, 4), "allgather_copy_s": round(t_copy, 4),
               "allgather_link_s": round(t_link, 4), "host_call_s": round(t_call, 4),
               "projected_rank_s": round(t_rank + t_copy + t_link + t_call, 4),
               "emulated_wall_s_not_a_projection": round(t_op, 4)}
        rows.append(row)
        print(json.dumps(row), flush=True)
ctx.close()
