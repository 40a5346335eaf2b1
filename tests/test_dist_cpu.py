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


class _FakeCtx:
    """Stands in for fhe_sign.Context: records what the fan-out control plane asks of it."""

    def __init__(self, fail=False, not_ready=False):
        self.fail, self.not_ready, self.calls = fail, not_ready, []

    def ready(self):
        if self.not_ready:
            raise RuntimeError("hipSetDevice failed")
        return True

    def attach_comm(self, uid, world, rank, timeout_ms=None):
        if self.fail:
            raise RuntimeError("attach refused")
        self.calls.append(("attach", uid, world, rank))

    def set_fanout(self, min_level):
        self.calls.append(("fanout", min_level))

    def detach_comm(self):
        self.calls.append(("detach",))


def _fanout_rank(rank, world, port, fail_rank, q, unready_rank=-1):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
    import torch.distributed as dist
    from fhe_sign.dist import attach_fanout
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = _FakeCtx(fail=rank == fail_rank, not_ready=rank == unready_rank)
    ok, err = attach_fanout(ctx, dist, rank, world, min_level=300, make_id=lambda: bytes(range(128)))
    q.put((rank, ok, ctx.calls))
    dist.destroy_process_group()


def _run_fanout(fail_rank, unready_rank=-1):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fanout_rank, args=(r, 2, port, fail_rank, q, unready_rank)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    return sorted(q.get() for _ in range(2))


def test_fanout_attach_world2_shares_rank0_id():
    """SURVEY 8e control plane: every rank attaches with rank 0's RCCL id and the split threshold."""
    got = _run_fanout(fail_rank=-1)
    for rank, ok, calls in got:
        assert ok
        assert calls == [("attach", bytes(range(128)), 2, rank), ("fanout", 300)]


def test_fanout_unready_rank_stops_everyone_before_the_init():
    """A rank that fails BEFORE the (collective) communicator init -- e.g. its device is unusable --
    is agreed on first: no rank calls attach_comm at all, so nobody waits in ncclCommInitRank for a
    peer that will never come (comm.cpp additionally bounds the init with a deadline)."""
    got = _run_fanout(fail_rank=-1, unready_rank=1)
    assert [(ok, calls) for _, ok, calls in got] == [(False, []), (False, [])]


def test_fanout_attach_failure_is_agreed():
    """one rank failing to attach makes every rank back out (no rank is left in a collective)"""
    got = _run_fanout(fail_rank=1)
    assert [ok for _, ok, _ in got] == [False, False]
    assert got[0][2][-1] == ("detach",)


class _KeyCtx:
    """fhe_sign.Context stand-in for the key-replication control plane."""

    def __init__(self, has_key):
        self.params = object() if has_key else None
        self.broadcasts = []

    def broadcast_server_key(self, root):
        self.broadcasts.append(root)


def _replicate_rank(rank, world, port, root_has_key, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
    import torch.distributed as dist
    from fhe_sign.dist import replicate_server_key
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = _KeyCtx(has_key=(rank == 0 and root_has_key))
    ok, err = replicate_server_key(ctx, dist, rank, root=0)
    q.put((rank, ok, ctx.broadcasts))
    dist.destroy_process_group()


def _run_replicate(root_has_key):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_replicate_rank, args=(r, 2, port, root_has_key, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    return sorted(q.get() for _ in range(2))


def test_server_key_replication_world2():
    """SURVEY 8e key replication: with a key on the root every rank enters the broadcast; without
    one, no rank enters the collective and all report failure (nobody waits alone)."""
    assert _run_replicate(True) == [(0, True, [0]), (1, True, [0])]
    assert [(r, ok, b) for r, ok, b in _run_replicate(False)] == [(0, False, []), (1, False, [])]


def test_fanout_deadline_guard():
    """bench.py's N > 1 fan-out legs run under a deadline: a hung leg is abandoned, not waited on."""
    import importlib.util
    import threading
    import time
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench.with_deadline(lambda: {"ok": 1}, 5.0) == ({"ok": 1}, False)
    r, hung = bench.with_deadline(lambda: 1 / 0, 5.0)
    assert not hung and "error" in r
    stop = threading.Event()
    t = time.perf_counter()
    r, hung = bench.with_deadline(lambda: stop.wait(30), 0.2)
    assert hung and r is None and time.perf_counter() - t < 5
    stop.set()


def test_fanout_hang_exits_nonzero():
    """A hung fan-out leg is abandoned AND the process exits with a non-zero status (3): the driver
    must record the run as failed, not as rc 0 with an 'error' buried in the JSON."""
    import subprocess
    code = (
        "import importlib.util, threading, json\n"
        f"spec = importlib.util.spec_from_file_location('b', {os.path.join(ROOT, 'bench.py')!r})\n"
        "b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)\n"
        "r, hung = b.with_deadline(lambda: threading.Event().wait(60), 0.2)\n"
        "print(json.dumps({'value': 1.0}), flush=True)\n"
        "if hung: b.abandon('test hang')\n"
    )
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert p.returncode == 3, (p.returncode, p.stderr)
    assert '"value": 1.0' in p.stdout and "status 3" in p.stderr


def _bare_env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env["HIP_VISIBLE_DEVICES"] = ""  # the launcher makes no GPU call; neither does a dry rank
    return env


def test_bare_gpus2_self_launches_and_relays_rank0_line():
    """`python bench.py --gpus 2` from a bare shell (no RANK/WORLD_SIZE): bench.py starts its own two
    ranks as child processes (never exec), they meet on gloo, and the launcher relays rank 0's one
    JSON line (n_gpus 2, max-over-ranks time) and exits 0."""
    import json
    import subprocess
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--dry-run"],
                       capture_output=True, text=True, timeout=180, env=_bare_env())
    assert p.returncode == 0, p.stderr
    lines = p.stdout.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout  # stdout: the one JSON line only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["dry_run"] and rec["steps"] == 3
    # max over ranks: rank 1 sleeps 0.1 s, so the whole-job step time reflects it
    assert rec["ms_per_step"] >= 0.1 / 3 * 1e3
    assert rec["pid"] != os.getpid()


def test_bare_launch_exits_nonzero_when_a_rank_fails():
    """A failing rank (status 5) makes the launcher exit non-zero; its peer, stuck in the barrier,
    is killed after the grace period instead of hanging the run."""
    import subprocess
    import time
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                        "--dry-fail-rank", "1"], capture_output=True, text=True, timeout=240, env=_bare_env())
    assert p.returncode == 5, (p.returncode, p.stderr)
    assert "exited with status 5" in p.stderr
    assert time.monotonic() - t0 < 200


def test_bare_launch_deadline_kills_every_rank():
    """The launcher's deadline kills ranks that never finish and returns 124."""
    import subprocess
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                        "--dry-fail-rank", "7", "--launch-deadline", "0.5"],
                       capture_output=True, text=True, timeout=120, env=_bare_env())
    assert p.returncode == 124, (p.returncode, p.stderr)
    assert "deadline" in p.stderr


def _transport_rank(rank, world, port, q):
    """the test transport's callbacks (tests/gloo_transport.py) called through their C function pointers,
    as comm.cpp calls them, on host buffers"""
    import ctypes as C
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import gloo_transport
    bcast, gather, amin = gloo_transport.callbacks(rank, world)
    out = {}
    buf = (C.c_uint8 * 1000)(*([7 if rank == 1 else 0] * 1000))
    assert bcast(None, C.addressof(buf), 1000, 1) == 0
    out["bcast"] = set(buf) == {7}
    seg = 4096
    g = (C.c_uint8 * (seg * world))()
    for k in range(seg):
        g[rank * seg + k] = (rank * 31 + k) % 251
    assert gather(None, C.addressof(g), seg) == 0
    out["gather"] = all(g[r * seg + k] == (r * 31 + k) % 251 for r in range(world) for k in range(seg))
    f = (C.c_uint8 * 64)(*[(k + rank) % 3 for k in range(64)])
    assert amin(None, C.addressof(f), 64) == 0
    out["min"] = list(f) == [min((k + r) % 3 for r in range(world)) for k in range(64)]
    q.put((rank, out))
    dist.destroy_process_group()


def test_test_transport_callbacks_world2():
    """The gloo test transport that stands in for RCCL in the one-GPU world-2 fan-out test
    (test_fanout_gpu.py::test_world2_fanout_gloo_transport): broadcast, all-gather of rank segments and
    the element-wise min, called through the same C function pointers the engine calls."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_transport_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    got = dict(q.get() for _ in range(2))
    assert got[0] == got[1] == {"bcast": True, "gather": True, "min": True}
