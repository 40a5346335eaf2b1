"""Multi-GPU fan-out control plane: one process per GPU.

The data path is the engine's own RCCL communicator (comm.cpp: in-place all-gather of each split
level on the engine stream).  This module only does the out-of-band part over an already
initialised torch.distributed process group (gloo is enough): rank 0 creates the RCCL id, every
rank receives it, the ranks agree that every one of them is ready BEFORE anyone enters the
communicator init (itself a collective), attach with a non-blocking init polled against a deadline
(comm.cpp: a peer that dies inside the init gives FHE_ERR_TIMEOUT, not a hang), and agree again that
all of them succeeded before any data-path collective is issued.
"""
from __future__ import annotations

from .core import comm_unique_id


def all_ok(dist, ok: bool) -> bool:
    """True iff `ok` holds on every rank (gloo all-reduce MIN)."""
    import torch
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def share_id(dist, rank: int, make_id=comm_unique_id) -> bytes | None:
    """Rank 0's RCCL unique id on every rank (None everywhere if rank 0 could not create one)."""
    import torch
    buf = torch.zeros(129, dtype=torch.uint8)
    if rank == 0:
        try:
            buf[:128] = torch.tensor(list(make_id()), dtype=torch.uint8)
            buf[128] = 1
        except Exception:  # noqa: BLE001 -- reported through the flag
            buf[128] = 0
    dist.broadcast(buf, 0)
    return bytes(buf[:128].tolist()) if int(buf[128]) else None


def attach_fanout(ctx, dist, rank: int, world: int, min_level: int = 257, make_id=comm_unique_id,
                  timeout_ms: int = 120000):
    """Attach `ctx` to a world-size RCCL communicator and enable level fan-out.
    Returns (ok, error): ok is identical on all ranks.

    1. rank 0's id is shared (None everywhere if it could not make one);
    2. every rank reports readiness (id received, context alive, device usable) and the ranks agree
       on it before the init: a rank that fails here makes nobody enter the collective;
    3. the init itself runs under `timeout_ms` (a peer dying inside it -> error on the others);
    4. the ranks agree that every attach succeeded, else all detach."""
    uid = share_id(dist, rank, make_id)
    ready, err = uid is not None, None
    if not ready:
        err = "rank 0 could not create an RCCL id"
    else:
        try:
            check_ready = getattr(ctx, "ready", None)
            ready = bool(check_ready()) if check_ready else True
            if not ready:
                err = f"rank {rank}: context/device not ready"
        except Exception as e:  # noqa: BLE001
            ready, err = False, f"rank {rank}: {e}"
    if not all_ok(dist, ready):
        return False, err or "another rank was not ready to attach"
    ok = True
    try:
        ctx.attach_comm(uid, world, rank, timeout_ms)
        ctx.set_fanout(min_level)
    except Exception as e:  # noqa: BLE001
        ok, err = False, str(e)
    if not all_ok(dist, ok):
        try:
            ctx.detach_comm()
        except Exception:  # noqa: BLE001
            pass
        return False, err or "another rank failed to attach"
    return True, None


def replicate_server_key(ctx, dist, rank: int, root: int = 0) -> tuple[bool, str | None]:
    """After attach_fanout: rank `root` (which called ctx.set_server_key) replicates its server key
    to every rank's context over RCCL (fhe_ctx_broadcast_server_key).  The ranks first agree that
    the root has a key, so nobody enters the collective alone.  Returns (ok, error) on every rank."""
    ok = rank != root or getattr(ctx, "params", None) is not None  # set by Context.set_server_key
    if not all_ok(dist, ok):
        return False, "the root rank has no server key"
    try:
        ctx.broadcast_server_key(root)
    except Exception as e:  # noqa: BLE001
        return False, str(e)
    return True, None
