"""Multi-GPU fan-out of the radix layer exercised on one GPU.

A fanned-out level is split into contiguous rank slices that bootstrap into a gather buffer, are
all-gathered (RCCL) and scattered into the block slots.  Here the split runs (a) over emulated
ranks on one device -- every slice is computed locally, so the outputs must be byte-identical to
the unsplit run, which pins the partition / gather / scatter indexing -- and (b) through a real
RCCL communicator of world 1 (the all-gather path with the library).  Multi-rank RCCL on distinct
GPUs is exercised by bench.py's fan-out leg at N > 1; the out-of-band id exchange is covered on
CPU by tests/test_dist_cpu.py."""
import csv
import json
import os
import random

import numpy as np
import pytest

from conftest import ROOT

from fhe_sign import (COMPAT, FAST, BigUintFHE, Context, FheUint64, FheUint256, Schnorr, comm_unique_id, compute_nonce,
                      generate_keys, set_server_key)

pytestmark = pytest.mark.gpu


def run_ops(ctx, ck):
    set_server_key(ctx)
    rng = random.Random(5)
    a, b = rng.getrandbits(256) | 1 << 255, rng.getrandbits(64)
    ck.seed_encryption(77)  # identical ciphertext inputs for every configuration
    A, B = FheUint256.try_encrypt(a, ck), FheUint64.try_encrypt(b, ck)
    outs = {
        "div": A / (rng.getrandbits(32) | 1),
        "mul64": B * FheUint64.try_encrypt(rng.getrandbits(64), ck),
        "sum": A + FheUint256.try_encrypt(rng.getrandbits(256), ck),
    }
    return {k: v.export() for k, v in outs.items()}, {k: v.decrypt(ck) for k, v in outs.items()}


@pytest.fixture(scope="module")
def keys():
    ck, sk = generate_keys(seed=0xFA11)
    return ck, sk


def test_emulated_ranks_byte_identical(keys):
    ck, sk = keys
    ref_ctx = Context(0)
    ref_ctx.set_server_key(sk)
    ref_ct, ref_val = run_ops(ref_ctx, ck)
    assert ref_ctx.fanout_info() == (0, 1, 0)
    for ranks in (2, 3, 8):
        ctx = Context(0)
        ctx.set_server_key(sk)
        ctx.set_fanout(min_level=1, emulate_ranks=ranks)
        ct, val = run_ops(ctx, ck)
        assert val == ref_val
        for k in ref_ct:
            assert np.array_equal(ct[k], ref_ct[k]), (ranks, k)
        _, world, split = ctx.fanout_info()
        assert world == ranks and split > 0
        ctx.close()
    set_server_key(None)
    ref_ctx.close()


def test_rccl_world1_all_gather(keys):
    ck, sk = keys
    ctx = Context(0)
    ctx.set_server_key(sk)
    ctx.attach_comm(comm_unique_id(), 1, 0)
    ctx.set_fanout(min_level=1)
    _, val = run_ops(ctx, ck)
    ref_ctx = Context(0)
    ref_ctx.set_server_key(sk)
    _, ref_val = run_ops(ref_ctx, ck)
    assert val == ref_val
    set_server_key(ctx)
    d, msg = 3, bytes(32)
    k0 = compute_nonce(d, msg, bytes(32))
    s = Schnorr()
    assert s.sign_fhe_with_k0(msg, k0, d, BigUintFHE.new(d, ck), ck, FAST) == s.sign_with_k0(msg, k0, d)
    ctx.detach_comm()
    set_server_key(None)
    ctx.close()
    ref_ctx.close()


def test_rccl_world1_server_key_broadcast(keys):
    """fhe_ctx_broadcast_server_key (the key replicated over xGMI) on a world-1 RCCL
    communicator: the root's key survives the collective bit for bit and keeps computing; misuse
    (no communicator, a root without a key) is refused.  The receiving side (ranks != root) needs a
    second GPU: it runs on the driver's multi-GPU node only."""
    ck, sk = keys
    ctx = Context(0)
    with pytest.raises(RuntimeError):
        ctx.broadcast_server_key(0)  # no communicator attached
    ctx.attach_comm(comm_unique_id(), 1, 0)
    with pytest.raises(RuntimeError):
        ctx.broadcast_server_key(0)  # root without a key
    ctx.set_server_key(sk)
    before = ctx.export_fourier_bsk()
    ctx.broadcast_server_key(0)
    assert np.array_equal(ctx.export_fourier_bsk().view(np.uint64), before.view(np.uint64))
    _, val = run_ops(ctx, ck)
    ref_ctx = Context(0)
    ref_ctx.set_server_key(sk)
    _, ref_val = run_ops(ref_ctx, ck)
    assert val == ref_val
    ctx.detach_comm()
    set_server_key(None)
    ctx.close()
    ref_ctx.close()


def _bcast_case(ctx, ck):
    """inputs of a fanned-out sign: a BigUintFHE private key (8 limbs) and a 256-bit FheUint whose
    upper blocks are trivial (cast up from 64 bits) -- both through the broadcast's receiving path"""
    set_server_key(ctx)
    d = int(CSV["1"]["secret key"], 16)
    D = BigUintFHE.new(d, ck)
    X = FheUint64.try_encrypt(0x0123_4567_89AB_CDEF, ck).cast_into(FheUint256)
    return d, D, X


@pytest.mark.parametrize("ranks", [0, 2])
def test_operand_broadcast_loopback(keys, ranks):
    """fhe_ctx_broadcast_biguint / _radix without a communicator (one GPU; `ranks` emulated): the
    root's blocks take the receiving path locally -- gather into one device buffer, metadata encode /
    validate, scatter into fresh slots -- so the copy's ciphertext words must equal the original's,
    trivial blocks stay trivial, and the copies compute: sign_fhe_with_k0 on the broadcast key ==
    the CSV (BIP-340 vector 1, src/schnorr.rs:270-277)."""
    ck, sk = keys
    ctx = Context(0)
    ctx.set_server_key(sk)
    if ranks:
        ctx.set_fanout(min_level=257, emulate_ranks=ranks)
    d, D, X = _bcast_case(ctx, ck)
    D2 = BigUintFHE.broadcast(D, 0, ctx)
    X2 = FheUint256.broadcast(X, 0, ctx)
    assert D2.handle.value != D.handle.value and X2.handle.value != X.handle.value
    for u, v in zip(D.digits, D2.digits):
        assert np.array_equal(u.export(), v.export())
    assert np.array_equal(X.export(), X2.export())
    assert X2.decrypt(ck) == 0x0123_4567_89AB_CDEF
    row = CSV["1"]
    msg, aux = bytes.fromhex(row["message"]), bytes.fromhex(row["aux_rand"])
    k0 = compute_nonce(d, msg, aux)
    sig = Schnorr().sign_fhe_with_k0(msg, k0, d, D2, ck, COMPAT)
    assert sig.hex().upper() == row["signature"].upper()
    with pytest.raises(RuntimeError):
        BigUintFHE.broadcast(D, 1 if ranks == 0 else ranks, ctx)  # root outside the world
    set_server_key(None)
    ctx.close()


def test_rccl_world1_operand_broadcast(keys):
    """the same collectives through a real RCCL communicator of world 1 (header, agreement
    all-reduce, metadata and ciphertext broadcasts, bounded wait): the root keeps its handle, and the
    context keeps computing afterwards.  The receiving side of a real communicator needs a second GPU
    (the driver's multi-GPU node); its code path is the loopback one above."""
    ck, sk = keys
    ctx = Context(0)
    ctx.set_server_key(sk)
    ctx.attach_comm(comm_unique_id(), 1, 0)
    d, D, X = _bcast_case(ctx, ck)
    assert BigUintFHE.broadcast(D, 0, ctx) is D
    assert FheUint256.broadcast(X, 0, ctx) is X
    assert D.to_biguint(ck) == d and X.decrypt(ck) == 0x0123_4567_89AB_CDEF
    ctx.detach_comm()
    set_server_key(None)
    ctx.close()


# ---------------------------------------------------------------- config 5 at the production split
CSV = {r["index"]: r for r in csv.DictReader(open(os.path.join(ROOT, "tests", "golden", "bip340_vectors.csv")))}
GOLD = os.path.join(ROOT, "tests", "golden")


def _limbs(x):
    return [int(v) for v in x]


def _config5(ctx, ck):
    """What config 5 runs (inputs via the operand broadcast): sign_fhe_with_k0 (compat, fast) on vector 0, its FHE block k + e*d' for
    vector 1 (8x8 limbs) as ciphertexts, the compat 256-bit mul, and the 8-sign batch of SURVEY 8d
    (vectors 0, 1, 2, 15, 16, 17, 18, 0).  Returns (ciphertext words, decrypted values)."""
    set_server_key(ctx)
    ck.seed_encryption(0xC5, 100)  # identical ciphertext inputs for every configuration
    s = Schnorr()
    g = json.load(open(os.path.join(GOLD, "biguint_vectors.json")))["mul"][0]
    v1 = json.load(open(os.path.join(GOLD, "sign_vectors.json")))["vectors"][1]
    val = lambda limbs: sum(int(x) << (32 * i) for i, x in enumerate(limbs))  # noqa: E731
    # the inputs through the operand broadcast (on one GPU its receiving path, locally), as a
    # fanned-out run receives them from rank 0
    bc = lambda v: BigUintFHE.broadcast(BigUintFHE.new(v, ck), 0, ctx)  # noqa: E731
    A, B = bc(val(g["a"])), bc(val(g["b"]))
    E, D, K = (bc(val(v1[k])) for k in ("e", "d", "k"))
    mul = A.mul(B, COMPAT)
    block = E.mul_add(D, K, COMPAT)
    cts = {"mul_compat": [x.export() for x in mul.digits], "sign_block_v1": [x.export() for x in block.digits]}
    vals = {"mul_compat": mul.decrypt_limbs(ck), "sign_block_v1": block.decrypt_limbs(ck)}
    d, msg = 3, bytes(32)
    k0 = compute_nonce(d, msg, bytes(32))
    dF = BigUintFHE.new(d, ck)
    vals["sign_v0_compat"] = s.sign_fhe_with_k0(msg, k0, d, dF, ck, COMPAT)
    vals["sign_v0_fast"] = s.sign_fhe_with_k0(msg, k0, d, dF, ck, FAST)
    jobs = []
    for idx in ("0", "1", "2", "15", "16", "17", "18", "0"):
        row = CSV[idx]
        dd = int(row["secret key"], 16)
        mm, aux = bytes.fromhex(row["message"]), bytes.fromhex(row["aux_rand"])
        jobs.append((mm, compute_nonce(dd, mm, aux), dd, BigUintFHE.new(dd, ck)))
    vals["batch8"] = s.sign_fhe_with_k0_batch(jobs, ck, COMPAT)
    return cts, vals, (g, v1)


@pytest.fixture(scope="module")
def config5_ref(keys):
    ck, sk = keys
    ctx = Context(0)
    ctx.set_server_key(sk)
    cts, vals, (g, v1) = _config5(ctx, ck)
    # the unsplit run itself against the reference's data
    assert vals["mul_compat"] == _limbs(g["out"])
    assert vals["sign_block_v1"] == _limbs(v1["sum"])
    assert vals["sign_v0_compat"].hex().upper() == CSV["0"]["signature"].upper()
    assert vals["sign_v0_fast"].hex().upper() == CSV["0"]["signature"].upper()
    for idx, sig in zip(("0", "1", "2", "15", "16", "17", "18", "0"), vals["batch8"]):
        assert sig.hex().upper() == CSV[idx]["signature"].upper(), idx
    set_server_key(None)
    ctx.close()
    return cts, vals


@pytest.mark.parametrize("ranks", [2, 4, 8])
def test_config5_emulated_ranks_production_split(keys, config5_ref, ranks):
    """config 5 (one sign / one 256-bit mul fanned over N GPUs, src/schnorr.rs:270-277) at the
    production split threshold (levels of >= 257 bootstraps, fhe_ctx_set_fanout's default): emulated
    ranks compute every slice on this GPU, so each ciphertext word must equal the unsplit run's, and
    every signature the CSV's (the 8-sign batch of SURVEY 8d included)."""
    ck, sk = keys
    ref_cts, ref_vals = config5_ref
    ctx = Context(0)
    ctx.set_server_key(sk)
    ctx.set_fanout(min_level=257, emulate_ranks=ranks)
    cts, vals, _ = _config5(ctx, ck)
    assert vals == ref_vals
    for k in ref_cts:
        assert len(cts[k]) == len(ref_cts[k])
        for x, y in zip(cts[k], ref_cts[k]):
            assert np.array_equal(x, y), (ranks, k)
    _, world, split = ctx.fanout_info()
    assert world == ranks and split > 0  # the compat mul's wide product levels were split
    set_server_key(None)
    ctx.close()


def test_rccl_world1_long_flush_keeps_progress(keys):
    """one flush of far more than 32 levels whose tail after the 32nd level takes longer
    than the deadline -- the 256-bit division by an encrypted divisor, ~870 dependent levels, ~2 s --
    completes under a 400 ms no-progress deadline: the outstanding progress marks are spread over
    the whole queue (fhe_ctx::mark_progress), not stuck at the 32nd level."""
    ck, sk = keys
    ctx = Context(0)
    ctx.set_server_key(sk)
    ctx.attach_comm(comm_unique_id(), 1, 0)
    set_server_key(ctx)
    a, d = (1 << 255) + 0x1234_5678_9ABC_DEF0_1357, (1 << 127) + 0xFEDC_BA98_7654_3210
    A, D = FheUint256.try_encrypt(a, ck), FheUint256.try_encrypt(d, ck)
    ctx.sync()
    ctx.set_comm_timeout(400)
    q, r = A.div_rem(D)
    ctx.sync()
    assert load_comm_attached(ctx)
    assert (q.decrypt(ck), r.decrypt(ck)) == (a // d, a % d)
    set_server_key(None)
    ctx.close()


def test_rccl_world1_sync_is_bounded(keys):
    """While a communicator is attached, fhe_ctx_sync waits through the bounded path
    (fhe_ctx::wait_stream), whose deadline counts time WITHOUT PROGRESS: (a) a compat 256-bit mul
    (~0.6 s over 151 levels, no level above ~0.25 s) completes under a 400 ms deadline, since every
    completed level restarts it (at world size 1 no dead-node agreement runs: that collective is for
    nranks > 1 only); (b) one raw 8192-PBS launch (one kernel, ~60 ms, no level marks) under a 2 ms
    deadline returns FHE_ERR_TIMEOUT with the communicator aborted and detached, and the context
    keeps computing afterwards."""
    from fhe_sign._lib import FHE_ERR_TIMEOUT, FheError
    ck, sk = keys
    ctx = Context(0)
    ctx.set_server_key(sk)
    with pytest.raises(FheError):
        ctx.set_comm_timeout(100)  # no communicator
    ctx.attach_comm(comm_unique_id(), 1, 0)
    set_server_key(ctx)
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "biguint_vectors.json")))["mul"][0]
    val = lambda limbs: sum(int(x) << (32 * i) for i, x in enumerate(limbs))  # noqa: E731
    A, B = BigUintFHE.new(val(g["a"]), ck), BigUintFHE.new(val(g["b"]), ck)
    ctx.set_comm_timeout(400)
    out = A.mul(B, COMPAT)
    ctx.sync()
    assert out.decrypt_limbs(ck) == _limbs(g["out"])
    assert ctx.fanout_info()[1] == 1 and load_comm_attached(ctx)
    # (b) no progress for longer than the deadline
    n = 8192
    lid = ctx.lut([(m + 1) % 16 for m in range(16)])
    cts = ck.encrypt_blocks(np.arange(n) % 16)
    d_in, d_out, d_lut = ctx.alloc(cts.nbytes), ctx.alloc(cts.nbytes), ctx.alloc(n * 4)
    ctx.h2d(d_in, cts)
    ctx.h2d(d_lut, np.full(n, lid, np.uint32))
    ctx.sync()
    ctx.set_comm_timeout(2)
    ctx.pbs_device(d_in, n, d_lut, d_out)
    with pytest.raises(FheError) as e:
        ctx.sync()
    assert e.value.code == FHE_ERR_TIMEOUT
    assert not load_comm_attached(ctx)  # aborted and detached
    ctx.sync()  # no communicator: a plain stream wait
    got = np.zeros_like(cts)
    ctx.d2h(got, d_out)
    assert all(ck.decrypt_block(got[i]) == (i % 16 + 1) % 16 for i in range(0, n, 97))
    for p in (d_in, d_out, d_lut):
        ctx.free(p)
    set_server_key(None)
    ctx.close()


def load_comm_attached(ctx) -> bool:
    """a communicator is attached (fhe_ctx_set_comm_timeout refuses otherwise)"""
    from fhe_sign._lib import FheError
    try:
        ctx.set_comm_timeout(120000)
        return True
    except FheError:
        return False


@pytest.mark.parametrize("world", [2, 4])
def test_world2_fanout_gloo_transport(world):
    """Config 5 readiness on one GPU: TWO processes run the production fan-out with real rank slices
    through the test transport (tests/fanout_gloo_rank.py, tests/gloo_transport.py; RCCL refuses two
    ranks per device): rank 1 receives the server key (broadcast_server_key's receive side) and the
    operands (broadcast_biguint); each rank bootstraps only its own slice of every split level; the
    dead-node all-reduce runs while rank 1 holds a handle rank 0 dropped.  The compat 256-bit product's
    ciphertext bytes are equal on both ranks and equal to the unsplit run's; fast mul, the extra node,
    both signers on BIP-340 vectors 0 and 1, the batch signer (tail flushes) and a 128-bit encrypted
    division (launch slices) are exact on both ranks."""
    import socket
    import subprocess
    import sys
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "fanout_gloo_rank.py")],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    res = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=420)
            assert p.returncode == 0, e[-3000:]
            res.append(json.loads(o.strip().splitlines()[-1]))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    res = sorted(res, key=lambda x: x["rank"])
    print(*(json.dumps(r) for r in res), sep="\n")
    for r in res:
        assert r["compat_ok"] and r["fast_ok"] and r["sig0_ok"] and r["sig1_ok"], res
        assert r["batch_ok"] and r["div_ok"], r
        assert r["compat_split_levels"] > 0 and r["split_levels"] > r["compat_split_levels"], r
        assert r["rank_pbs"] < r["pbs"], r  # each rank bootstrapped only its slices of the split levels
        assert r["compat_sha"] == res[0]["unsplit_sha"], r
    assert all(r["extra_ok"] for r in res[1:])
    assert res[0]["unsplit_ok"]
