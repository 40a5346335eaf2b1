"""Diagnostic of the world-2 test-transport fan-out (tests/fanout_gloo_rank.py): which ops / split
settings give wrong results.  usage: python3 tools/fanout_gloo_diag.py   (launches its own 2 ranks)"""
import json
import os
import random
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rank_main():
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ref_semantics as R
    from fhe_sign import COMPAT, FAST, BigUintFHE, Context, generate_keys, set_server_key
    import gloo_transport
    ck, sk = generate_keys(seed=0x6A11)
    ctx = Context(0)
    ctx.set_server_key(sk)
    set_server_key(ctx)
    rng = random.Random(9)
    res = []
    for min_level in (1 << 30, 257):
        gloo_transport.attach(ctx, rank, world, min_level=min_level)
        for la, lb in ((2, 2), (3, 3), (8, 2), (8, 8)):
            a = [rng.getrandbits(32) for _ in range(la)]
            b = [rng.getrandbits(32) for _ in range(lb)]
            ck.seed_encryption(1000 + la * 10 + lb, 100)
            A, B = BigUintFHE.new(R.from_limbs(a), ck), BigUintFHE.new(R.from_limbs(b), ck)
            _, _, lv0 = ctx.fanout_info()
            got = A.mul(B, COMPAT).decrypt_limbs(ck)
            _, _, lv1 = ctx.fanout_info()
            fast = A.mul(B, FAST).to_biguint(ck) == R.from_limbs(a) * R.from_limbs(b)
            res.append({"min_level": min_level, "shape": [la, lb], "compat_ok": got == R.biguint_mul(a, b),
                        "fast_ok": fast, "split": lv1 - lv0})
        ctx.detach_comm()
    print(json.dumps({"rank": rank, "res": res}), flush=True)
    dist.barrier()
    set_server_key(None)
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    if "RANK" in os.environ:
        rank_main()
        sys.exit(0)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)],
                              env=dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                                       MASTER_PORT=str(port))) for r in range(2)]
    codes = [p.wait(timeout=300) for p in procs]
    sys.exit(max(codes))
