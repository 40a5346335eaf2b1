"""Per-node output hashes (FHE_DEBUG=nodes) of a 2x2 compat BigUintFHE mul: the world-2 test-transport
split on both ranks, then on rank 0 the emulated split and the unsplit run on the same inputs.  Writes
gpurun_out/diag2_rank{r}.log.  usage: python3 tools/fanout_gloo_diag2.py"""
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rank_main():
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    for d in ("fhe-sign_amd", "tests", "oracle"):
        sys.path.insert(0, os.path.join(ROOT, d))
    import ref_semantics as R
    from fhe_sign import COMPAT, BigUintFHE, Context, generate_keys, set_server_key
    import gloo_transport
    ck, sk = generate_keys(seed=0x6A11)
    ctx = Context(0)
    ctx.set_server_key(sk)
    set_server_key(ctx)
    a, b = [0x89ABCDEF, 0x12345678], [0xFEDCBA98, 0x0F0F0F0F]
    ck.seed_encryption(77, 100)
    A, B = BigUintFHE.new(R.from_limbs(a), ck), BigUintFHE.new(R.from_limbs(b), ck)
    want = R.biguint_mul(a, b)
    A.add(B).to_biguint(ck)  # LUT registration / pools outside the logged part
    gloo_transport.attach(ctx, rank, world, min_level=257)
    print("=== real", flush=True, file=sys.stderr)
    got = A.mul(B, COMPAT).decrypt_limbs(ck)
    print(f"=== real ok={got == want}", flush=True, file=sys.stderr)
    dist.barrier()
    ctx.detach_comm()
    if rank == 0:
        ctx.set_fanout(257, 2)
        print("=== emulated", flush=True, file=sys.stderr)
        got = A.mul(B, COMPAT).decrypt_limbs(ck)
        print(f"=== emulated ok={got == want}", flush=True, file=sys.stderr)
        ctx.set_fanout(257, 0)
        print("=== unsplit", flush=True, file=sys.stderr)
        got = A.mul(B, COMPAT).decrypt_limbs(ck)
        print(f"=== unsplit ok={got == want}", flush=True, file=sys.stderr)
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
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    logs = [open(os.path.join(ROOT, "gpurun_out", f"diag2_rank{r}.log"), "w") for r in range(2)]
    procs = [subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)], stderr=logs[r],
                              env=dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                                       MASTER_PORT=str(port), FHE_DEBUG="nodes")) for r in range(2)]
    codes = [p.wait(timeout=300) for p in procs]
    sys.exit(max(codes))
