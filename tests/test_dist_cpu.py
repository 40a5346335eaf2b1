"""N>1 control plane of bench.py on CPU: world_size-2 gloo ranks, barrier + max-over-ranks timing,
per-rank replica seeding (weak scaling, no data-path collective; DESIGN.md 'Multi-GPU')."""
import os
import socket
import sys

import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    sys.path.insert(0, ROOT)
    import bench
    dist, r, w, local = bench.dist_setup(world)
    assert (r, w, local) == (rank, world, rank)
    bench.barrier(dist)
    m = bench.allmax(dist, float(rank + 1) * 1.5)
    q.put((rank, m))
    dist.destroy_process_group()


def test_bench_control_plane_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    got = sorted(q.get() for _ in range(2))
    assert got == [(0, 3.0), (1, 3.0)]  # every rank sees the max over ranks


def test_single_rank_needs_no_process_group():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.dist_setup(1) == (None, 0, 1, 0)
    assert bench.allmax(None, 2.5) == 2.5
