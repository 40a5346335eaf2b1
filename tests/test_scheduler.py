"""The radix engine's level scheduler (csrc/radix.cpp:schedule_levels, C ABI fhe_schedule_levels),
host logic only: on random dependency graphs and on the shape of a compat window-add chain, every
node runs after its inputs, the level count is the critical path, levels are filled to whole
latency-kernel rounds (256) only with work that could run there, and the backward schedule keeps
the throughput work off the chain levels' critical capacity."""
import ctypes as C
import os
import random

import numpy as np
import pytest

from fhe_sign import _lib


def schedule(deps, mode=0, ranks=1):
    n = len(deps)
    off = np.zeros(n + 1, np.int32)
    for i, d in enumerate(deps):
        off[i + 1] = off[i] + len(d)
    flat = np.array([x for d in deps for x in d] or [0], np.int32)
    level = np.zeros(max(n, 1), np.int32)
    nl = C.c_int32()
    P = C.POINTER(C.c_int32)
    rc = _lib.load().fhe_schedule_levels_ranks(off.ctypes.data_as(P), flat.ctypes.data_as(P), n, mode, ranks,
                                               level.ctypes.data_as(P), C.byref(nl))
    assert rc == 0, _lib.load().fhe_last_error()
    return level[:n].tolist(), nl.value


def critical_path(deps):
    d = []
    for i, ds in enumerate(deps):
        d.append(1 + max((d[j] for j in ds), default=0))
    return max(d, default=0)


def check(deps, level, nl):
    assert nl == critical_path(deps)
    for i, ds in enumerate(deps):
        assert 1 <= level[i] <= nl
        for j in ds:
            assert level[j] < level[i], (i, j)


@pytest.mark.parametrize("mode", [0, 1])
def test_random_graphs(mode):
    rng = random.Random(7 + mode)
    for trial in range(30):
        n = rng.randrange(1, 3000)
        deps = []
        for i in range(n):
            k = rng.choice([0, 0, 1, 2, 3, 6]) if i else 0
            deps.append(sorted(set(rng.randrange(0, i) for _ in range(min(k, i)))))
        level, nl = schedule(deps, mode)
        check(deps, level, nl)


def test_chain_with_background_work():
    """A 100-level chain of 64-node steps beside 20000 independent two-stage jobs each needed by
    one chain step: the level count stays the chain's, the chain levels are filled to one round
    (256), and what does not fit runs early in large levels (backward schedule)."""
    deps, prev = [], []
    jobs = []
    for j in range(20000):  # stage 1, then stage 2 reading it
        deps.append([])
        deps.append([len(deps) - 1])
        jobs.append(len(deps) - 1)
    for step in range(100):
        cur = []
        for k in range(64):
            d = list(prev[max(0, k - 2):k + 1]) + [jobs[(step * 200 + k) % len(jobs)]]
            deps.append(sorted(set(d)))
            cur.append(len(deps) - 1)
        prev = cur
    level, nl = schedule(deps, 0)
    check(deps, level, nl)
    sizes = np.bincount(level, minlength=nl + 1)[1:]
    assert nl == 102
    assert (sizes[5:] <= 256).all() and (sizes[5:] >= 200).sum() > 80  # chain levels filled to a round
    assert sizes[:2].sum() > 20000  # the rest as large early batches
    lf, nf = schedule(deps, 1)
    check(deps, lf, nf)


FANOUT_MIN = 257  # bench.py / fhe_ctx_set_fanout default: levels of at least this many bootstraps are split


def chain_graph(steps=100, width=64, jobs_n=20000):
    deps, prev, jobs = [], [], []
    for j in range(jobs_n):
        deps.append([])
        deps.append([len(deps) - 1])
        jobs.append(len(deps) - 1)
    for step in range(steps):
        cur = []
        for k in range(width):
            d = list(prev[max(0, k - 2):k + 1]) + [jobs[(step * 200 + k) % len(jobs)]]
            deps.append(sorted(set(d)))
            cur.append(len(deps) - 1)
        prev = cur
    return deps


@pytest.mark.parametrize("ranks", [2, 4, 8])
def test_fanout_partition_divides_the_fill(ranks):
    """The fan-out partition (config 5a) on the chain-with-background graph, as the engine's flush runs
    it over N ranks (levels filled to one latency round PER RANK, 256 N): the level count stays the
    chain's; the 40000 off-chain bootstraps ride inside the chain levels, the filled ones reach the
    split threshold and are divided over the ranks, so no rank's slice of any level exceeds one round:
    the op takes exactly as many latency rounds as the chain has levels (the 1-GPU schedule needs ~80
    more rounds for the fill).  Levels below the threshold -- the chain plus fill that cannot move later
    -- run redundantly: one round either way, so splitting them would only add a collective."""
    deps = chain_graph()
    level, nl = schedule(deps, 0, ranks)
    check(deps, level, nl)
    assert nl == 102
    sizes = np.bincount(level, minlength=nl + 1)[1:]
    assert (sizes <= 256 * ranks).all()
    split = sizes >= FANOUT_MIN
    per_rank = [(-(-int(g) // ranks) if s else int(g)) for g, s in zip(sizes, split)]
    assert max(per_rank) <= 256  # every level is one latency round on every rank
    rounds = sum(-(-p // 256) for p in per_rank)
    assert rounds == nl  # every level is one round on every rank: the chain's floor
    assert sum(per_rank) < len(deps) * 0.6  # each rank runs well under the whole graph
    l1, n1 = schedule(deps, 0, 1)
    assert n1 == nl
    rounds1 = sum(-(-int(g) // 256) for g in np.bincount(l1, minlength=n1 + 1)[1:])
    assert rounds1 > nl + 70


def test_invalid_graph_rejected():
    off = np.array([0, 1], np.int32)
    bad = np.array([0], np.int32)  # node 0 reading itself
    level = np.zeros(1, np.int32)
    nl = C.c_int32()
    P = C.POINTER(C.c_int32)
    assert _lib.load().fhe_schedule_levels(off.ctypes.data_as(P), bad.ctypes.data_as(P), 1, 0,
                                           level.ctypes.data_as(P), C.byref(nl)) != 0


def test_progress_marks_stay_spread():
    """with up to 32 progress marks outstanding, a flush of L levels that the
    GPU has not started keeps marks spread over the whole queue -- the largest gap between
    consecutive outstanding marks stays within ~2x the mean (L / 32), so a long healthy flush shows
    progress at least every ~L/16 levels instead of going silent after its 32nd level."""
    import ctypes
    for levels, bound in ((10, 1), (32, 1), (33, 2), (149, 10), (869, 60), (5000, 330)):
        gap = ctypes.c_uint32()
        assert _lib.load().fhe_progress_marks_probe(levels, ctypes.byref(gap)) == 0
        assert 1 <= gap.value <= bound, (levels, gap.value)


_FP_SCRIPT = r"""
import ctypes, random, sys
sys.path.insert(0, sys.argv[1])
from fhe_sign import _lib
libc = ctypes.CDLL(None)
libc.malloc.restype = ctypes.c_void_p
rng = random.Random(int(sys.argv[2]))
keep = [libc.malloc(rng.randrange(16, 1 << 16)) for _ in range(rng.randrange(0, 4000))]  # shift the C++ heap
out = []
for la, lb, lk, mode in ((2, 2, 0, 0), (8, 8, 0, 0), (8, 8, 0, 1), (8, 1, 8, 0), (3, 5, 0, 0)):
    fp = ctypes.c_uint64()
    assert _lib.load().fhe_host_biguint_mul_fingerprint(la, lb, lk, mode, ctypes.byref(fp)) == 0
    out.append(fp.value)
    keep += [libc.malloc(rng.randrange(16, 1 << 12)) for _ in range(rng.randrange(0, 500))]
print(out)
"""


def test_recording_order_is_address_independent():
    """The fan-out splits a level by position and every rank scatters the gathered slices by ITS node
    order, so every rank must record the same graph in the same order.  Three processes with differently
    perturbed C++ heaps record the BigUintFHE mul (compat and fast, 2x2 to 8x8, the signer's mul-add) and
    must produce equal recording-order fingerprints (Engine::fingerprint: no addresses).  Round 6 found
    the Karatsuba half sums walked in operand-address order (the world-2 GPU test's wrong compat limbs)."""
    import subprocess
    import sys
    from conftest import ROOT
    outs = []
    for seed in (1, 2, 3):
        r = subprocess.run([sys.executable, "-c", _FP_SCRIPT, os.path.join(ROOT, "fhe-sign_amd"), str(seed)],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(r.stdout.strip())
    assert outs[0] == outs[1] == outs[2], outs
