"""One rank of the world-2 fan-out test on ONE GPU (tests/test_fanout_gpu.py::test_world2_fanout_gloo_
transport; not collected by pytest).  Both ranks share device 0 and exchange through the test transport
(tests/gloo_transport.py) -- the production split with real rank slices:
  * ranks >= 1 have no server key: they receive rank 0's over fhe_ctx_broadcast_server_key (the receive side:
    fresh buffers, ksk_to_planes, bsk_to_e on a non-root rank);
  * the operands exist on rank 0 only and reach the others through fhe_ctx_broadcast_biguint;
  * every level of >= 257 bootstraps is split, each rank bootstrapping only its own slice, outputs
    all-gathered; dead nodes agreed by the min all-reduce while ranks >= 1 hold a handle rank 0 dropped;
  * compat / fast 256-bit mul and sign_fhe_with_k0 (BIP-340 vectors 0 and 1, fused and call-site forms),
    the batch signer and a 128-bit encrypted division (launched in slices).
Rank 0 then detaches and recomputes the compat product alone: the serialized ciphertext words of the
split run (both ranks) must equal the unsplit run's.  Prints one JSON line per rank."""
import csv
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    from fhe_sign import (COMPAT, FAST, BigUintFHE, Context, FheUint128, Schnorr, compute_nonce, generate_keys,
                          rank_pbs, set_server_key, stats)
    import gloo_transport
    out = {"rank": rank}
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "biguint_vectors.json")))["mul"][0]
    val = lambda limbs: sum(int(x) << (32 * i) for i, x in enumerate(limbs))  # noqa: E731
    a, b = val(golden["a"]), val(golden["b"])
    rows = {r["index"]: r for r in csv.DictReader(open(os.path.join(ROOT, "tests", "golden", "bip340_vectors.csv")))}
    ck, sk = generate_keys(seed=0x6A11)  # the same client key on both ranks (decryption checks)
    ctx = Context(0)
    if rank == 0:
        ctx.set_server_key(sk)
    gloo_transport.attach(ctx, rank, world, min_level=257)
    ctx.broadcast_server_key(0)
    set_server_key(ctx)
    ck.seed_encryption(0x5EED, 100)
    A, B = (BigUintFHE.broadcast(BigUintFHE.new(v, ck) if rank == 0 else None, 0, ctx) for v in (a, b))
    # a node only ranks >= 1 keep alive: rank 0 drops its handle before the next flush, so the dead-node
    # agreement (min over the ranks) must keep it on both
    extra = A.add(B, FAST)
    if rank == 0:  # only the other ranks keep it
        del extra
    _, _, lv0 = ctx.fanout_info()
    P = A.mul(B, COMPAT)
    out["compat_ok"] = P.decrypt_limbs(ck) == [int(x) for x in golden["out"]]
    _, _, lv1 = ctx.fanout_info()
    out["compat_split_levels"] = lv1 - lv0
    out["compat_sha"] = hashlib.sha256(P.serialize()).hexdigest()
    if rank >= 1:
        out["extra_ok"] = extra.to_biguint(ck) == a + b  # graph empty: a local read
    out["fast_ok"] = A.mul(B, FAST).to_biguint(ck) == a * b
    s = Schnorr()
    sigs = {}
    for idx in ("0", "1"):
        d = int(rows[idx]["secret key"], 16)
        msg, aux = bytes.fromhex(rows[idx]["message"]), bytes.fromhex(rows[idx]["aux_rand"])
        k0 = compute_nonce(d, msg, aux)
        dF = BigUintFHE.broadcast(BigUintFHE.new(d, ck) if rank == 0 else None, 0, ctx)
        sigs[idx] = [s.sign_fhe_with_k0(msg, k0, d, dF, ck, COMPAT).hex().upper(),
                     s.sign_fhe_with_k0_callsite(msg, k0, d, dF, ck, COMPAT).hex().upper()]
        out[f"sig{idx}_ok"] = sigs[idx] == [rows[idx]["signature"].upper()] * 2
    # the batch signer (each signature's products launched as recorded: Engine::flush_tail) and a
    # 128-bit encrypted division deep enough to launch in slices (flush_depth), both split over the ranks
    jobs, want = [], []
    for idx in ("0", "1"):
        d = int(rows[idx]["secret key"], 16)
        msg, aux = bytes.fromhex(rows[idx]["message"]), bytes.fromhex(rows[idx]["aux_rand"])
        jobs.append((msg, compute_nonce(d, msg, aux), d, BigUintFHE.broadcast(BigUintFHE.new(d, ck) if rank == 0 else None, 0, ctx)))
        want.append(bytes.fromhex(rows[idx]["signature"]))
    out["batch_ok"] = s.sign_fhe_with_k0_batch(jobs, ck, COMPAT) == want
    x, y = (a >> 128) | 1, (b & ((1 << 64) - 1)) | (1 << 63)
    X, Y = (FheUint128.broadcast(FheUint128.try_encrypt(v, ck) if rank == 0 else None, 0, ctx) for v in (x, y))
    qo, ro = X.div_rem(Y)
    out["div_ok"] = (qo.decrypt(ck), ro.decrypt(ck)) == (x // y, x % y)
    _, _, lv2 = ctx.fanout_info()
    out["split_levels"] = lv2
    out["rank_pbs"], out["pbs"] = rank_pbs(ctx), stats(ctx)[0]
    dist.barrier()
    ctx.detach_comm()
    if rank == 0:  # the unsplit run on the same input ciphertexts
        P1 = A.mul(B, COMPAT)
        out["unsplit_sha"] = hashlib.sha256(P1.serialize()).hexdigest()
        out["unsplit_ok"] = P1.decrypt_limbs(ck) == [int(x) for x in golden["out"]]
    print(json.dumps(out), flush=True)
    dist.barrier()
    set_server_key(None)
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
