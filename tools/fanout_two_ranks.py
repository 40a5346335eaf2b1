"""Two ranks on whatever GPUs are visible (torch.distributed gloo for the RCCL id, one process per
rank): fanned-out BigUintFHE mul + sign must equal the single-process result.  With one GPU both
ranks share device 0 (RCCL may refuse that; the error is reported).
usage: python3 tools/fanout_two_ranks.py"""
import os, sys
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))


def worker(rank, world, port, q):
    import random
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fhe_sign import FAST, BigUintFHE, Context, comm_unique_id, generate_keys, set_server_key
        import torch
        ndev = torch.cuda.device_count()
        ck, sk = generate_keys(seed=0xFA11)
        ctx = Context(rank % max(1, ndev)); ctx.set_server_key(sk); set_server_key(ctx)
        uid = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            uid = torch.tensor(list(comm_unique_id()), dtype=torch.uint8)
        dist.broadcast(uid, 0)
        ctx.attach_comm(bytes(uid.tolist()), world, rank)
        ctx.set_fanout(min_level=256)
        rng = random.Random(3)
        a, b = rng.getrandbits(256), rng.getrandbits(256)
        ck.seed_encryption(11)
        A, B = BigUintFHE.new(a, ck), BigUintFHE.new(b, ck)
        r = A.mul(B, FAST).to_biguint(ck)
        q.put((rank, r == a * b, ctx.fanout_info()))
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        q.put((rank, f"error: {e}", None))
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    mp.set_start_method("spawn")
    q = mp.Queue()
    ps = [mp.Process(target=worker, args=(r, 2, 29517, q)) for r in range(2)]
    for p in ps: p.start()
    for p in ps: p.join(240)
    res = [q.get(timeout=5) for _ in ps if not q.empty()]
    print(res, flush=True)
    sys.exit(0 if len(res) == 2 and all(r[1] is True for r in res) else 1)
