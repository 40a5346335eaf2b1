"""Test-only transport (fhe_ctx_attach_test_transport, include/fhe_rocm.h) over a gloo process group:
several ranks on ONE GPU run the production fan-out -- each computes only its own slice of a split
level, the outputs are all-gathered, dead nodes agreed by a min all-reduce, keys and operands
broadcast -- with the collectives host-staged through torch.distributed instead of RCCL (which
refuses two ranks per device).  Never used by the product: bench.py and fhe_sign.dist use RCCL."""
import ctypes as C
import sys
import traceback

from fhe_sign import _lib


def _view(addr, nbytes):
    import torch
    return torch.frombuffer((C.c_uint8 * nbytes).from_address(addr), dtype=torch.uint8)


def callbacks(rank: int, world: int):
    """the three C callbacks (bcast, allgather, allreduce_min_u8) over the default process group"""
    import torch
    import torch.distributed as dist

    def guarded(fn):
        def call(*args):
            try:
                fn(*args)
                return 0
            except Exception:  # noqa: BLE001 -- reported to the engine as a failed collective
                traceback.print_exc(file=sys.stderr)
                return 1
        return call

    def bcast(user, host, nbytes, root):
        dist.broadcast(_view(host, nbytes), src=root)

    def allgather(user, host, seg):
        t = _view(host, seg * world)
        parts = list(t.split(seg))
        outs = [torch.empty(seg, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(outs, parts[rank].clone())
        for r in range(world):
            if r != rank:
                parts[r].copy_(outs[r])

    def amin(user, host, n):
        t = _view(host, n)
        x = t.to(torch.int32)
        dist.all_reduce(x, op=dist.ReduceOp.MIN)
        t.copy_(x.to(torch.uint8))

    return _lib.TX_BCAST(guarded(bcast)), _lib.TX_ALLGATHER(guarded(allgather)), _lib.TX_MIN_U8(guarded(amin))


def attach(ctx, rank: int, world: int, min_level: int = 257):
    """attach the gloo transport to `ctx` and enable the level fan-out; returns the transport object
    (keep it referenced while attached: it owns the callbacks)"""
    cbs = callbacks(rank, world)
    tx = _lib.TestTransport(None, *cbs)
    _lib.check(_lib.load().fhe_ctx_attach_test_transport(ctx.handle, C.byref(tx), world, rank))
    ctx.set_fanout(min_level)
    ctx._test_transport = (tx, cbs)  # the engine holds the function pointers while attached
    return tx
