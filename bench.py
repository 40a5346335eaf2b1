#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X-native TFHE engine.

Metric (BASELINE.json): "PBS/s + 256-bit FHE mul wall-clock; sign_fhe_with_k0 seconds".
A step = one batch of `--batch` programmable bootstraps (KS -> MS -> BR -> SE) over big-key LWE
blocks already resident in HBM, i.e. one DAG level of the radix ops that BigUintFHE::mul issues
(src/biguint.rs:223; the widest level of a 256-bit 8x8-limb mul is thousands of block PBS).
`value` = PBS per second over all ranks.  Ranks are independent replicas of the batch
(weak scaling; the path has no exchange step, so no data-path collective).

Timed region: barrier + device sync, K steps, device sync + barrier; max over ranks.
roofline: the dominant kernel (blind rotate) timed live with HIP events on the engine's stream;
algorithmic f64 flops per PBS = n * 2^18, peak = FP64 vector rate.
cpu_baseline: the C oracle (same algorithm, same parameters) on host cores, rank 0, N=1 only.
"""
from __future__ import annotations

import argparse
import json
import threading
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))

import numpy as np  # noqa: E402

METRIC = "PBS/s + 256-bit FHE mul wall-clock; sign_fhe_with_k0 seconds @1/2/4/8 GPU"
FP64_PEAK_TFLOPS = 78.6        # MI355X dense FP64 peak (matrix = vector on gfx950), spec
FP64_PEAK_MEASURED_TFLOPS = 65.0  # dependent-free v_fma_f64 stream on the GPU box (tools/fp64_peak.hip)
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r6", "r6f_pmc_summary.json")  # tools/profile_round.sh (final r6 tree)
FANOUT_MIN = 257  # levels with at least this many bootstraps are split over the GPUs (fan-out legs)
OPS_REPS = 3  # timed runs per ops leg (median reported)
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
FLOPS_PER_CMUX = 4 * 51200 + 4 * 6144 + 32768   # 4 FFT-1024 (5 N log N), 4 twist/untwist, MAC
# multi-bit (grouping 2), per pair of key bits: the same transforms and MAC, plus the key bundle --
# per Fourier point 3 monomials minus 1 (3) and 3 patterns x 4 polynomials of complex multiply-add (96)
FLOPS_PER_GROUP_MB = FLOPS_PER_CMUX + 1024 * (3 + 96)
L2_PEAK_GBS = 34500.0          # MI355X_MICROARCH.md: L2 ~34.5 TB/s aggregate
CUS = 256                      # MI355X compute units
DETAIL_DEFAULT = os.path.join(ROOT, "profiles", "r6", "bench_detail_latest.json")
LINE_MAX_BYTES = 6144          # the driver keeps the last 8 KB of stdout; the line stays well inside it


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    # 32768 = the widest PBS level of configs[1]'s compat 256-bit mul (the first level: every block
    # product of the 8x8 limb products, profiles/r2/level_trace_r2c.txt), 42.7 rounds of the
    # throughput kernel's 768 resident workgroups
    ap.add_argument("--batch", type=int, default=32768, help="PBS per step per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample length")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--detail", default=DETAIL_DEFAULT,
                    help="side file for the per-run arrays, the multi-bit op legs and the CPU per-op replay")
    ap.add_argument("--seed", type=int, default=0xF11E51)
    ap.add_argument("--no-ops", action="store_true", help="skip the 256-bit mul / sign wall-clock legs")
    ap.add_argument("--no-multibit", action="store_true", help="skip the multi-bit (grouping 2) measurement")
    ap.add_argument("--launch-deadline", type=float, default=LAUNCH_DEADLINE_S,
                    help="self-launched N > 1 runs: seconds before every rank is killed")
    # GPU-free rehearsal of the N > 1 control plane (the launcher test): every rank joins the gloo
    # group, times a barrier-bracketed sleep, takes the max over ranks, rank 0 prints the line
    ap.add_argument("--dry-run", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--dry-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    return ap.parse_args(argv)


# ------------------------------------------------------------------------------------ launcher
LAUNCH_DEADLINE_S = 1500.0
LAUNCH_GRACE_S = 30.0  # after one rank fails, how long the others get to finish before being killed
LAUNCH_FAIL_EXIT = 4


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(n: int, argv: list, deadline_s: float) -> int:
    """`--gpus N > 1` started from a bare shell (no RANK/WORLD_SIZE in the environment): this process
    becomes the launcher.  It makes no GPU call (nothing here imports torch or the engine); it starts
    N rank processes of this same script as children -- subprocess, never exec -- each with
    RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT set, relays rank 0's stdout (the JSON line)
    and returns non-zero if any rank fails (its first failing status, or LAUNCH_FAIL_EXIT for a
    signal), killing the rest after LAUNCH_GRACE_S; at `deadline_s` every rank still running is
    killed and the launcher returns 124.  Under torchrun (WORLD_SIZE set) this is never reached."""
    import signal
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr, start_new_session=True))

    def relay():
        for line in procs[0].stdout:
            sys.stdout.write(line.decode(errors="replace"))
            sys.stdout.flush()

    th = threading.Thread(target=relay, daemon=True)
    th.start()

    def kill_all():
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except OSError:
                    pass
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                pass

    t_end = time.monotonic() + deadline_s
    failed_at, status = None, 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad and failed_at is None:
            failed_at = time.monotonic()
            status = bad[0] if bad[0] > 0 else LAUNCH_FAIL_EXIT
            sys.stderr.write(f"bench launcher: a rank exited with status {bad[0]}\n")
        if all(c is not None for c in codes):
            break
        now = time.monotonic()
        if now > t_end:
            sys.stderr.write(f"bench launcher: deadline of {deadline_s:.0f} s passed; killing every rank\n")
            kill_all()
            th.join(5)
            return 124
        if failed_at is not None and now - failed_at > LAUNCH_GRACE_S:
            sys.stderr.write("bench launcher: killing the ranks left after a failure\n")
            kill_all()
            break
        time.sleep(0.2)
    th.join(10)
    return status


def dry_run(a, dist, rank, world, out):
    """The N > 1 control plane without a GPU: barrier + sleep + barrier, max over ranks, one line."""
    if rank == a.dry_fail_rank:
        sys.stderr.write(f"bench dry run: rank {rank} failing on request\n")
        sys.exit(5)
    barrier(dist)
    t0 = time.perf_counter()
    time.sleep(0.05 * (rank + 1))
    dt = allmax(dist, time.perf_counter() - t0)
    barrier(dist)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": world * a.steps / dt, "unit": "steps/s (dry run)",
                          "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": dt / a.steps * 1e3,
                          "dry_run": True, "pid": os.getpid()}), file=out, flush=True)
    if dist is not None:
        dist.destroy_process_group()


def dist_setup(n):
    if n <= 1 and int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return None, 0, 1, 0
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("gloo")  # control plane only (barrier, max of times)
    return dist, dist.get_rank(), dist.get_world_size(), int(os.environ.get("LOCAL_RANK", "0"))


def barrier(dist):
    if dist is not None:
        dist.barrier()


def allmax(dist, x: float) -> float:
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def host_cores():
    """(threads to use, description): every CPU this process may run on (sched_getaffinity), capped by
    the cgroup CPU quota when one is set (on the GPU box the affinity mask can show the whole
    machine while the container's share is smaller); nproc reported beside it."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    threads = aff if quota is None else max(1, min(aff, int(round(quota))))
    return threads, {"nproc": os.cpu_count(), "affinity": aff, "cgroup_cpu_quota": quota}


# ops whose launched levels are replayed through the C restatement (measured), and ops whose CPU time
# is projected from the measured per-PBS time level by level (too long to replay in a default run)
CPU_REPLAY_OPS = ("biguint256_add_fast", "sign_fhe_with_k0_v0_compat", "sub256", "shr256_encrypted", "and256")
CPU_PROJECT_OPS = ("biguint256_mul_compat", "biguint256_mul_fast", "sign_fhe_v0_compat", "div256_by_u32")


def cpu_baseline(seed, target_s, op_levels=None):
    """The CPU restatement (oracle/tfhe_oracle.c, bit-exact with the GPU path; NOT tfhe-rs, which is
    absent) on this host's cores: PBS/s on a bounded sample, then the radix ops of configs 1, 2 and 4
    at the same levels the GPU engine launched (fhe_ctx_level_log): each level's bootstraps run as
    one OpenMP batch, so an op costs sum over levels of ceil(PBS_l / threads) rounds."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    threads, info = host_cores()
    ok = oracle.OracleKeys(seed)
    lut = ok.make_lut([(m + 1) % 16 for m in range(16)])[None, :]
    r = ok.rng(3)
    # calibrate with one PBS per thread, then size the sample to ~target_s
    cts = np.stack([ok.encrypt(r, m % 16) for m in range(threads)])
    t0 = time.perf_counter()
    ok.pbs_batch(cts, lut, np.zeros(threads, np.uint32), threads)
    per_round = time.perf_counter() - t0
    rounds = max(1, int(target_s / max(per_round, 1e-3)))
    count = threads * rounds
    pool = np.concatenate([cts] * rounds)
    t0 = time.perf_counter()
    ok.pbs_batch(pool, lut, np.zeros(count, np.uint32), threads)
    dt = time.perf_counter() - t0
    res = {"value": count / dt, "unit": "PBS/s", "cores": threads, "kind": "port", **info,
           "simd": {0: "scalar", 1: "avx2", 2: "avx512"}[int(oracle.load().fho_simd())],
           "sample": f"{count} PBS (KS+BR+SE, same params/keys shape) with the C oracle (bit-exact "
                     f"restatement; its blind rotation and keyswitch loops in AVX2 / AVX-512, bit-identical "
                     f"to their scalar form -- not tfhe-rs's FFT), OpenMP {threads} threads = every CPU of "
                     f"this process's affinity/cgroup share, {dt:.1f} s"}
    t_round = dt / rounds  # one round = `threads` bootstraps in parallel

    def rounds_of(sizes):
        return sum((n + threads - 1) // threads for n in sizes)

    ops = {}
    for name in CPU_REPLAY_OPS:
        sizes = (op_levels or {}).get(name)
        if not sizes:
            continue
        t0 = time.perf_counter()
        for n in sizes:
            batch = pool[:n] if n <= len(pool) else np.resize(pool, (n, pool.shape[1]))
            ok.pbs_batch(np.ascontiguousarray(batch), lut, np.zeros(n, np.uint32), threads)
        ops[name] = {"seconds": time.perf_counter() - t0, "how": "replayed", "pbs": sum(sizes), "levels": len(sizes),
                     "projected_seconds": rounds_of(sizes) * t_round}
    for name in CPU_PROJECT_OPS:
        sizes = (op_levels or {}).get(name)
        if sizes:
            ops[name] = {"seconds": rounds_of(sizes) * t_round, "how": "projected", "pbs": sum(sizes),
                         "levels": len(sizes)}
    if ops:
        res["ops"] = ops
        res["ops_note"] = (f"CPU restatement (oracle/tfhe_oracle.c), not tfhe-rs: each op's GPU-launched levels "
                           f"(level sizes from fhe_ctx_level_log) as OpenMP batches on {threads} threads "
                           f"(nproc {info['nproc']}); 'replayed' ran every bootstrap, 'projected' = sum over "
                           f"levels of ceil(PBS/threads) x the measured {t_round * 1e3:.1f} ms per round of "
                           f"{threads} bootstraps")
    return res


def pmc_traffic(batch, kernels=("k_blind_rotate_qy2<1>",)):
    """HBM-side bytes per launch of the blind-rotate kernel at this batch, from the committed PMC
    summary of the same kernel (tools/profile_round.sh; FETCH_SIZE x2 + WRITE_SIZE, gfx950
    correction of MI355X_MICROARCH.md 'HBM'; Infinity-Cache hits included).  `kernels`: name
    patterns tried in order (the classic kernel is the <1> instance of br_qy.hip's template; summaries
    from before it was a template name it without the argument)"""
    try:
        d = json.load(open(PMC_SUMMARY))["pmc"][f"B={batch}"]
        for kernel in kernels:
            k = next((v for k, v in d.items() if kernel in k), None)
            if k is not None:
                return k["hbm_side_bytes_per_launch"], os.path.relpath(PMC_SUMMARY, ROOT)
        return None, None
    except (OSError, KeyError, ValueError):
        return None, None


def golden_mul():
    """(a, b, compat limbs) of the first committed 8x8-limb vector (tests/golden/biguint_vectors.json,
    seeded 256-bit operands; `out` = the reference's limb loop src/biguint.rs:194-265, lost carries
    included): the legs check results against committed data, never against oracle code."""
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "biguint_vectors.json")))["mul"][0]
    val = lambda limbs: sum(int(x) << (32 * i) for i, x in enumerate(limbs))  # noqa: E731
    return val(g["a"]), val(g["b"]), [int(x) for x in g["out"]]


def ops_legs(ck, ctx, seed):
    """configs 2 and 4: BigUintFHE 256-bit mul wall-clock and sign_fhe_with_k0 seconds (every rank
    runs its own replica: the N-GPU line is the 'one sign per GPU' batch of configs[4])."""
    import random
    from fhe_sign import (COMPAT, FAST, PUBLIC, BigUintFHE, FheUint8, FheUint32, FheUint256, Schnorr, compute_nonce,
                          level_log, set_server_key, stats)
    set_server_key(ctx)
    rng = random.Random(seed)
    a, b, compat_limbs = golden_mul()
    A, B = BigUintFHE.new(a, ck), BigUintFHE.new(b, ck)
    out, level_sizes = {}, {}

    def leg(name, fn, check, reps=OPS_REPS):
        """reps timed runs (each result checked); seconds = the median, the level sizes of the last
        run kept for the CPU replay (cpu_baseline)"""
        runs = []
        for _ in range(reps):
            level_log(ctx)  # reset the per-level record
            p0, l0 = stats(ctx)
            t0 = time.perf_counter()
            r = fn()
            ctx.sync()
            runs.append(time.perf_counter() - t0)
            p1, l1 = stats(ctx)
            sizes = level_log(ctx)
            if not check(r):
                raise SystemExit(f"bench: {name} result mismatch")
        out[name] = {"seconds": float(np.median(runs)), "runs": runs, "pbs": p1 - p0, "levels": l1 - l0}
        level_sizes[name] = sizes

    A.add(B, FAST)  # warm-up (LUT registration, pools)
    A.mul(B, COMPAT).decrypt_limbs(ck)  # grows the block pool / staging buffers to their steady-state size
    leg("biguint256_mul_compat", lambda: A.mul(B, COMPAT), lambda r: r.decrypt_limbs(ck) == compat_limbs)
    leg("biguint256_mul_fast", lambda: A.mul(B, FAST), lambda r: r.to_biguint(ck) == a * b)
    leg("biguint256_add_fast", lambda: A.add(B, FAST), lambda r: r.to_biguint(ck) == a + b)
    # config 3: 256-bit radix / clear divisor (src/perf_test.rs:54 at 256 bits)
    A256 = FheUint256.try_encrypt(a, ck)
    du32, du128 = rng.getrandbits(32) | 1 << 31, rng.getrandbits(128) | 1 << 127
    leg("div256_by_5", lambda: A256 / 5, lambda r: r.decrypt(ck) == a // 5)
    leg("div256_by_u32", lambda: A256 / du32, lambda r: r.decrypt(ck) == a // du32)
    leg("div256_by_u128", lambda: A256 / du128, lambda r: r.decrypt(ck) == a // du128)
    # the stretch case of config 3: 256-bit by an ENCRYPTED 128-bit-valued divisor, quotient + remainder
    D256 = FheUint256.try_encrypt(du128, ck)
    leg("div256_by_encrypted", lambda: A256.div_rem(D256),
        lambda r: (r[0].decrypt(ck), r[1].decrypt(ck)) == (a // du128, a % du128))
    # north_star's other 256-bit ops (sub, encrypted shift, and; the reference applies them at 32 bits,
    # src/perf_test.rs:36,48; shift amount mod the width, src/biguint.rs:494-498)
    B256 = FheUint256.try_encrypt(b, ck)
    m256 = (1 << 256) - 1
    sh = rng.randrange(256)
    S256 = FheUint256.try_encrypt(sh, ck)
    cl256 = rng.getrandbits(256)
    leg("sub256", lambda: A256 - B256, lambda r: r.decrypt(ck) == (a - b) & m256)
    leg("shr256_encrypted", lambda: A256 >> S256, lambda r: r.decrypt(ck) == a >> sh)
    leg("shl256_encrypted", lambda: A256 << S256, lambda r: r.decrypt(ck) == (a << sh) & m256)
    leg("and256", lambda: A256 & B256, lambda r: r.decrypt(ck) == a & b)
    leg("and256_clear", lambda: A256 & cl256, lambda r: r.decrypt(ck) == a & cl256)
    X32 = FheUint32.try_encrypt(1344, ck)  # src/perf_test.rs:14-15,54 (README.md:114: 1121 s on CPU)
    leg("fheuint32_div5", lambda: X32 / 5, lambda r: r.decrypt(ck) == 268)
    leg("fheuint32_add", lambda: X32 + FheUint32.try_encrypt(5, ck), lambda r: r.decrypt(ck) == 1349)
    leg("fheuint32_mul", lambda: X32 * FheUint32.try_encrypt(5, ck), lambda r: r.decrypt(ck) == 6720)
    # the rest of src/perf_test.rs:36-48 (README.md:110-113): 1344 >> Enc(5) = 42, cast to u8, min with
    # Enc(7u8), & 1 -- each timed alone on its own inputs, like the reference's Instant pairs
    B5 = FheUint32.try_encrypt(5, ck)
    leg("fheuint32_shr_encrypted", lambda: X32 >> B5, lambda r: r.decrypt(ck) == 42)
    # each leg's input is computed (and read back: the engine defers work until a host read) before
    # its clock starts, so a leg times only its own operation
    S42 = X32 >> B5
    assert S42.decrypt(ck) == 42
    leg("fheuint32_cast_u8", lambda: S42.cast_into(FheUint8), lambda r: r.decrypt(ck) == 42)
    C8, C7 = S42.cast_into(FheUint8), FheUint8.try_encrypt(7, ck)
    assert C8.decrypt(ck) == 42
    leg("fheuint8_min", lambda: C8.min(C7), lambda r: r.decrypt(ck) == 7)
    M7 = C8.min(C7)
    assert M7.decrypt(ck) == 7
    leg("fheuint8_and1", lambda: M7 & 1, lambda r: r.decrypt(ck) == 1)
    d, msg = 3, bytes(32)  # BIP-340 vector 0 (tests/golden/bip340_vectors.csv row 0)
    k0 = compute_nonce(d, msg, bytes(32))
    dF = BigUintFHE.new(d, ck)
    s = Schnorr()
    ref = s.sign_with_k0(msg, k0, d)
    leg("sign_fhe_with_k0_v0_compat", lambda: s.sign_fhe_with_k0(msg, k0, d, dF, ck, COMPAT), lambda r: r == ref)
    # the reference's unchanged call site (src/schnorr.rs:271-276), operator by operator through the C
    # ABI as INTEGRATION.md 2's impl Add / impl Mul binding dispatches it: BigUintFHE::new(e), ::new(k),
    # k_fhe + (e_fhe * privkey_fhe) (normalized limbs), to_biguint, % n
    leg("sign_fhe_with_k0_v0_callsite", lambda: s.sign_fhe_with_k0_callsite(msg, k0, d, dF, ck, COMPAT),
        lambda r: r == ref)
    leg("sign_fhe_with_k0_v0_fast", lambda: s.sign_fhe_with_k0(msg, k0, d, dF, ck, FAST), lambda r: r == ref)
    leg("sign_fhe_with_k0_v0_public", lambda: s.sign_fhe_with_k0(msg, k0, d, dF, ck, PUBLIC), lambda r: r == ref)
    # Schnorr::sign_fhe (src/schnorr.rs:154-211): the full signer, encrypting the private key itself --
    # what README.md:104's 4269 s most likely measures
    import csv
    rows = {r["index"]: r for r in csv.DictReader(open(os.path.join(ROOT, "tests", "golden", "bip340_vectors.csv")))}
    csv0 = bytes.fromhex(rows["0"]["signature"])
    leg("sign_fhe_v0_compat", lambda: s.sign_fhe(msg, bytes(32), d, ck, COMPAT), lambda r: r == ref == csv0)
    # config 5b's batch on one GPU: 8 signatures (BIP-340 vectors 0, 1, 2, 15, 16, 17, 18, 0; SURVEY
    # 8d) as ONE engine schedule; signs/s = 8 / seconds
    jobs, want = [], []
    for idx in ("0", "1", "2", "15", "16", "17", "18", "0"):
        dd = int(rows[idx]["secret key"], 16)
        mm, aux = bytes.fromhex(rows[idx]["message"]), bytes.fromhex(rows[idx]["aux_rand"])
        kk = compute_nonce(dd, mm, aux)
        jobs.append((mm, kk, dd, BigUintFHE.new(dd, ck)))
        want.append(s.sign_with_k0(mm, kk, dd))
    leg("sign_fhe_with_k0_batch8_compat", lambda: s.sign_fhe_with_k0_batch(jobs, ck, COMPAT), lambda r: r == want)
    out["sign_fhe_with_k0_batch8_compat"]["signs_per_s"] = 8 / out["sign_fhe_with_k0_batch8_compat"]["seconds"]
    return out, level_sizes


FANOUT_DEADLINE_S = 180.0
FANOUT_HUNG_EXIT = 3


def with_deadline(fn, seconds):
    """fn() on a daemon thread: (result, timed_out).  The fan-out legs are the only part of the N > 1
    run that depends on RCCL between GPUs; if they hang, the measured line is still printed."""
    box = {}

    def run():
        try:
            box["r"] = fn()
        except Exception as e:  # noqa: BLE001 -- reported in the line
            box["r"] = {"error": str(e)}

    th = threading.Thread(target=run, daemon=True)
    th.start()
    th.join(seconds)
    return box.get("r"), th.is_alive()


def abandon(why):
    """End a run whose watchdog abandoned a GPU leg: the JSON line (already printed) is kept, but the
    process exits non-zero, so the run is recorded as failed -- never as a clean rc 0."""
    sys.stdout.flush()
    sys.stderr.write(f"bench: {why}; exiting with status {FANOUT_HUNG_EXIT}\n")
    sys.stderr.flush()
    os._exit(FANOUT_HUNG_EXIT)


def fanout_legs(ck, ctx, dist, rank, world, seed):
    """config 5 / SURVEY.md 8e: ONE 256-bit mul and ONE sign fanned across all ranks (levels of at
    least FANOUT_MIN bootstraps split over the GPUs, outputs all-gathered with RCCL).  Identical
    inputs on every rank; a failure on any rank stops the fan-out legs on all of them."""
    from fhe_sign import COMPAT, FAST, BigUintFHE, Schnorr, compute_nonce, set_server_key
    from fhe_sign.dist import all_ok, attach_fanout
    out = {"ranks": world, "min_level": FANOUT_MIN}
    ok, err = attach_fanout(ctx, dist, rank, world, min_level=FANOUT_MIN)
    if not ok:
        out["error"] = err
        return out
    set_server_key(ctx)
    a, b, compat_limbs = golden_mul()
    d, msg = 3, bytes(32)
    k0 = compute_nonce(d, msg, bytes(32))
    # The encrypted inputs exist on rank 0 only -- as sign_fhe_with_k0's privkey_fhe arrives from its
    # caller (src/schnorr.rs:235) -- and reach the other ranks device to device (RCCL broadcast,
    # fhe_ctx_broadcast_biguint): every rank then runs the program on byte-identical ciphertexts.
    ck.seed_encryption(seed ^ 0x5EED, 100)
    try:
        A, B, dF = (BigUintFHE.broadcast(BigUintFHE.new(v, ck) if rank == 0 else None, 0, ctx) for v in (a, b, d))
        good, why = True, None
    except Exception as e:  # noqa: BLE001 -- the collective agreed on the failure; reported below
        good, why = False, f"operand broadcast: {e}"
    if not all_ok(dist, good):
        out["error"] = why or "operand broadcast failed on another rank"
        return out
    s = Schnorr()
    ref = s.sign_with_k0(msg, k0, d)
    legs = [
        ("warmup_add_fast", lambda: A.add(B, FAST), lambda r: r.to_biguint(ck) == a + b),
        ("biguint256_mul_fast", lambda: A.mul(B, FAST), lambda r: r.to_biguint(ck) == a * b),
        ("biguint256_mul_compat", lambda: A.mul(B, COMPAT), lambda r: r.decrypt_limbs(ck) == compat_limbs),
        ("sign_fhe_with_k0_v0_compat", lambda: s.sign_fhe_with_k0(msg, k0, d, dF, ck, COMPAT), lambda r: r == ref),
        ("sign_fhe_with_k0_v0_fast", lambda: s.sign_fhe_with_k0(msg, k0, d, dF, ck, FAST), lambda r: r == ref),
    ]
    for name, fn, check in legs:
        barrier(dist)
        ctx.sync()
        _, _, lv0 = ctx.fanout_info()
        t0 = time.perf_counter()
        good, why = False, None
        try:
            r = fn()
            ctx.sync()
            dt = time.perf_counter() - t0
            good = bool(check(r))
            why = None if good else "result mismatch"
        except Exception as e:  # noqa: BLE001 -- agreed below, reported in the JSON line
            dt, why = time.perf_counter() - t0, str(e)
        _, _, lv1 = ctx.fanout_info()
        agreed = all_ok(dist, good)
        out[name] = {"seconds": allmax(dist, dt), "ok": agreed, "split_levels": lv1 - lv0}
        if not agreed:
            out["error"] = why or "failed on another rank"
            break
    try:
        ctx.detach_comm()
    except Exception:  # noqa: BLE001
        pass
    return out


def pbs_leg(a, kind, dist, rank, world, device):
    """one parameter set: keys, the timed batch of `a.batch` PBS per GPU (barrier + sync around exactly
    a.steps steps, max over ranks), the live HIP-event kernel timing and a decryption spot check.
    Returns (ck, ctx, result dict); the caller frees nothing (ctx.close() at exit)."""
    from fhe_sign import Context, default_params, generate_keys, multi_bit_params

    P = multi_bit_params() if kind == "multibit" else default_params()
    ck, sk = generate_keys(P, seed=a.seed)
    ctx = Context(device)
    ctx.set_server_key(sk)
    n = sk.params.lwe_dimension
    lid = ctx.lut([(m + 1) % 16 for m in range(16)])
    B = a.batch
    ck.seed_encryption(a.seed + rank, 100)
    # B distinct encryptions (distinct masks, hence distinct monomial-table gathers per step)
    cts = ck.encrypt_blocks(np.arange(B) % 16)
    d_in = ctx.alloc(cts.nbytes)
    d_out = ctx.alloc(cts.nbytes)
    d_lut = ctx.alloc(B * 4)
    ctx.h2d(d_in, cts)
    ctx.h2d(d_lut, np.full(B, lid, np.uint32))

    def latency_levels():
        """the latency kernel at the level sizes of the serial carry chains (one ciphertext per CU):
        best of 3 blind-rotate times (HIP events) at B = 1 and 256 -- the per-level floor of the
        compat mul / sign"""
        lat = {}
        ctx.enable_timing(True)
        for nb in (1, 256):
            ctx.pbs_device(d_in, nb, d_lut, d_out)  # untimed first launch (code object, workspace)
            best = 1e9
            for _ in range(3):
                ctx.pbs_device(d_in, nb, d_lut, d_out)
                best = min(best, ctx.last_pbs_timing()[1])
            lat[f"B={nb}"] = best
        ctx.enable_timing(False)
        return lat

    # before any throughput launch (cool chip) and again after the timed steps (clock under load):
    # both in the line, so a difference between them is the clock, measured in the same run
    lat_before = latency_levels()

    for _ in range(a.warmup):
        ctx.pbs_device(d_in, B, d_lut, d_out)
    ctx.sync()

    # live per-kernel timing (HIP events on the engine stream) in separate untimed passes
    ctx.enable_timing(True)
    ks_t, br_t = [], []
    for _ in range(max(2, min(a.steps, 5))):
        ctx.pbs_device(d_in, B, d_lut, d_out)
        ks, br = ctx.last_pbs_timing()
        ks_t.append(ks)
        br_t.append(br)
    ctx.enable_timing(False)
    ctx.sync()

    # shader clock over the timed steps: every workgroup of the blind rotate adds its lifetime in
    # s_memtime cycles and s_memrealtime 100 MHz ticks (fhe_ctx_enable_clock; two stamps per workgroup)
    ctx.enable_clock(True)
    barrier(dist)
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ctx.pbs_device(d_in, B, d_lut, d_out)
    ctx.sync()
    dt = time.perf_counter() - t0
    barrier(dist)
    dt = allmax(dist, dt)
    cycles, ticks, wgs = ctx.read_clock()
    ctx.enable_clock(False)

    # host-buffer boundary (fhe_pbs_batch: H2D + KS/BR + D2H), reported beside `value`, never as it
    t0 = time.perf_counter()
    host_reps = 2
    for _ in range(host_reps):
        ctx.pbs(cts, lid)
    pcie_rate = host_reps * B / (time.perf_counter() - t0)

    lat = {"before_throughput": lat_before, "after_throughput": latency_levels()}
    # correctness spot check of the last step (decrypt a sample)
    ctx.pbs_device(d_in, B, d_lut, d_out)
    out = np.zeros_like(cts)
    ctx.d2h(out, d_out)
    ok = all(ck.decrypt_block(out[i]) == (i % 16 + 1) % 16 for i in range(0, B, max(1, B // 64)))
    if not ok:
        raise SystemExit(f"bench: decryption check failed ({kind})")
    for d in (d_in, d_out, d_lut):
        ctx.free(d)

    br_ms = float(np.mean(br_t))
    ks_ms = float(np.mean(ks_t))
    flops_pbs = n * FLOPS_PER_CMUX if kind == "classic" else n // 2 * FLOPS_PER_GROUP_MB
    achieved = B * flops_pbs / (br_ms * 1e-3) / 1e12
    ggsw = n if kind == "classic" else n // 2 * 3
    bsk_bytes = ggsw * 4 * 1024 * 16
    # algorithmic HBM bytes of one blind-rotate launch: the Fourier BSK once, per PBS the keyswitched
    # LWE u64[n + 1] in, the big LWE u64[2049] out and its u32 LUT index
    hbm_bytes = bsk_bytes + B * ((n + 1) * 8 + 2049 * 8 + 4)
    # every workgroup streams the whole Fourier BSK from L2 (classic: k_blind_rotate_qy2, two ciphertexts
    # per workgroup sharing it; multi-bit: one per workgroup): the bytes the blind rotate moves L2 -> CU
    # per launch, and their rate against the L2 peak
    l2_bytes = ((B + 1) // 2 if kind == "classic" else B) * bsk_bytes
    res = {
        "value": world * B * a.steps / dt,
        "ms_per_step": dt / a.steps * 1e3,
        "params": f"n={n},N=2048,k=1,pbs=2^23x1,ks=2^3x5,msg=4,carry=4,grouping={1 if kind == 'classic' else 2}",
        "roofline": {
            "bound": "fp64_valu",
            "compute_pipe": "fp64 VALU (FFT butterflies; no dense contraction on the path)",
            "kernel": "k_blind_rotate_qy2<1>" if kind == "classic" else "k_blind_rotate_qy<2>",
            "achieved": achieved,
            "peak": FP64_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved / FP64_PEAK_TFLOPS,
            "peak_measured": FP64_PEAK_MEASURED_TFLOPS,
            "frac_measured": achieved / FP64_PEAK_MEASURED_TFLOPS,
            "flops_per_pbs": flops_pbs,
            "kernel_ms": br_ms,
            "keyswitch_ms": ks_ms,
            "hbm": {"bound": "hbm", "achieved": hbm_bytes / (br_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": hbm_bytes / (br_ms * 1e-3) / 1e9 / HBM_PEAK_GBS},
            "l2": {"bound": "l2_to_cu", "achieved": l2_bytes / (br_ms * 1e-3) / 1e9, "peak": L2_PEAK_GBS,
                   "unit": "GB/s", "frac": l2_bytes / (br_ms * 1e-3) / 1e9 / L2_PEAK_GBS,
                   "bytes_per_launch": l2_bytes},
        },
        "pcie_inclusive_pbs_per_s": pcie_rate * world,  # per-rank host-buffer rate x ranks
        "latency_level_ms": lat,
    }
    if ticks and wgs:
        ghz = cycles / ticks * 0.1  # s_memrealtime counts at 100 MHz
        res["clock"] = {
            "shader_ghz": ghz,
            # clock-normalised cost (drift between boxes is clock): CU-cycles per bootstrap of the timed
            # step (KS + BR + SE) and of the blind rotate alone (HIP-event kernel time)
            "cu_cycles_per_pbs": res["ms_per_step"] * 1e-3 * ghz * 1e9 * CUS / B,
            "br_cu_cycles_per_pbs": br_ms * 1e-3 * ghz * 1e9 * CUS / B,
            "wg_cycles": cycles / wgs,  # one workgroup's lifetime (classic: two ciphertexts), shader cycles
            "workgroups": wgs,
            "source": "s_memtime / s_memrealtime of every blind-rotate workgroup over the timed steps",
        }
    return ck, ctx, res


def _sig(x, digits=5):
    """floats to `digits` significant digits, recursively (the line stays short)"""
    if isinstance(x, float):
        return float(f"{x:.{digits}g}")
    if isinstance(x, dict):
        return {k: _sig(v, digits) for k, v in x.items()}
    if isinstance(x, list):
        return [_sig(v, digits) for v in x]
    return x


# published reference CPU numbers for the same operations (README.md:104-114; c5.24xlarge,
# likely a debug build) -- context only, in the detail file
README_S = {"fheuint32_add": 25.965747001, "fheuint32_mul": 76.051254698, "fheuint32_div5": 1121.134781795,
            "fheuint32_shr_encrypted": 45.566019345, "fheuint32_cast_u8": 135.023e-6, "fheuint8_min": 25.71097148,
            "fheuint8_and1": 6.418014644, "sign_fhe_v0_compat": 4269.0}
# the classic (default-parameter) headline keys, emitted LAST so that the driver's stdout tail keeps them
HEADLINE_KEYS = ("biguint256_mul_seconds", "biguint256_mul_fast_seconds", "sign_fhe_with_k0_seconds",
                 "sign_fhe_with_k0_callsite_seconds", "div256_seconds", "div256_by_encrypted_seconds",
                 "latency_level_ms")
# multi-bit summary keys -> its op legs
MB_KEYS = (("biguint256_mul_seconds", "biguint256_mul_compat"), ("biguint256_mul_fast_seconds", "biguint256_mul_fast"),
           ("sign_fhe_with_k0_seconds", "sign_fhe_with_k0_v0_compat"),
           ("sign_fhe_with_k0_callsite_seconds", "sign_fhe_with_k0_v0_callsite"),
           ("div256_by_encrypted_seconds", "div256_by_encrypted"))


def compose_line(a, world, cl, ops, mb, fan, cpu):
    """(the one JSON line, the detail dict).  The line: the contract keys, compact roofline / clock /
    multi-bit / fan-out / CPU-baseline summaries, every classic op's median seconds, then HEADLINE_KEYS
    last (< LINE_MAX_BYTES; tests/test_bench_line.py).  The detail (side file, a.detail): the per-run
    arrays, the reference-equivalent op/s, the README comparison, the multi-bit op legs and the CPU
    per-op replay."""
    B = a.batch
    traffic, traffic_src = pmc_traffic(B, (cl["roofline"]["kernel"],))
    r = cl["roofline"]
    roof = {k: r[k] for k in ("bound", "kernel", "achieved", "peak", "unit", "frac", "peak_measured", "frac_measured",
                              "flops_per_pbs", "kernel_ms", "keyswitch_ms")}
    roof["traffic"] = traffic
    roof["traffic_source"] = traffic_src
    roof["hbm"] = {k: r["hbm"][k] for k in ("achieved", "peak", "unit", "frac")}
    roof["l2_to_cu"] = {k: r["l2"][k] for k in ("achieved", "peak", "unit", "frac")}
    res = {
        "metric": METRIC,
        "value": cl["value"],
        "unit": "PBS/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": cl["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": f"batched PBS (KS+MS+BR+SE) of {B} 2_2 radix blocks per GPU (configs[1]: 32768 = the "
                        "block products of the 256-bit BigUintFHE mul, 128x128 pairs x lo/hi)",
            "batch_pbs_per_gpu": B,
            "params": cl["params"],
            "parallelism": f"replicas x{world}",
        },
        "roofline": roof,
    }
    if "clock" in cl:
        res["clock"] = {k: v for k, v in cl["clock"].items() if k != "source"}
    res["pcie_inclusive_pbs_per_s"] = cl["pcie_inclusive_pbs_per_s"]
    detail = {"metric": METRIC, "roofline": r, "clock": cl.get("clock"), "latency_level_ms": cl["latency_level_ms"]}
    if mb is not None:
        t_mb, _ = pmc_traffic(B, ("k_blind_rotate_qy<2>",))
        m = {"value": mb["value"], "ms_per_step": mb["ms_per_step"], "kernel": mb["roofline"]["kernel"],
             "frac": mb["roofline"]["frac"], "kernel_ms": mb["roofline"]["kernel_ms"], "traffic": t_mb}
        if "clock" in mb:
            m["shader_ghz"] = mb["clock"]["shader_ghz"]
            m["cu_cycles_per_pbs"] = mb["clock"]["cu_cycles_per_pbs"]
        m["latency_level_ms"] = mb["latency_level_ms"]
        if "ops" in mb:
            for key, leg in MB_KEYS:
                if leg in mb["ops"]:
                    m[key] = mb["ops"][leg]["seconds"]
            detail["multibit_ops"] = mb["ops"]
        res["multibit"] = m
        detail["multibit"] = {k: v for k, v in mb.items() if k != "ops"}
    if fan is not None:
        res["fanout"] = fan
    if cpu is not None:
        c = {k: cpu[k] for k in ("value", "unit", "cores", "kind", "simd", "nproc", "cgroup_cpu_quota") if k in cpu}
        c["sample"] = (cpu["sample"].split(" (")[0] + " with the C restatement oracle/tfhe_oracle.c (not tfhe-rs), "
                       f"{cpu['cores']} OpenMP threads")
        if "ops" in cpu:
            c["ops_s"] = {k: v["seconds"] for k, v in cpu["ops"].items()}
        res["cpu_baseline"] = c
        detail["cpu_baseline"] = cpu
    res["detail"] = os.path.relpath(os.path.abspath(a.detail), ROOT) if a.detail else None
    if ops is not None:
        res["ops_s"] = {k: v["seconds"] for k, v in ops.items()}
        detail["ops"] = ops
        # reference-equivalent op/s (the reference's operations per second on one GPU)
        detail["reference_equivalent_ops_per_s"] = {k: 1.0 / v["seconds"] for k, v in ops.items() if v["seconds"] > 0}
        detail["vs_reference_readme"] = {k: {"reference_s": v, "this_s": ops[k]["seconds"],
                                             "speedup": v / ops[k]["seconds"]} for k, v in README_S.items() if k in ops}
        res["ops_pbs_levels"] = {k: [ops[k]["pbs"], ops[k]["levels"]] for _, k in MB_KEYS if k in ops}
        for key, leg in MB_KEYS[:4]:
            res[key] = ops[leg]["seconds"]
        res["div256_seconds"] = ops["div256_by_u32"]["seconds"]
        res["div256_by_encrypted_seconds"] = ops["div256_by_encrypted"]["seconds"]
    # blind rotate of one latency level, B = 1 / 256, before and after the timed throughput steps
    res["latency_level_ms"] = cl["latency_level_ms"]
    return _sig(res), detail


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # bare `python bench.py --gpus N`: be the launcher (no GPU call in this process)
        sys.exit(self_launch(a.gpus, sys.argv[1:], a.launch_deadline))
    # stdout carries exactly the one JSON line: libraries that print banners there (RCCL prints its
    # version block at communicator init) are sent to stderr instead
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    sys.stdout = sys.stderr
    dist, rank, world, local = dist_setup(a.gpus)
    if a.dry_run:
        dry_run(a, dist, rank, world, out)
        return

    device = local
    if dist is not None:  # more ranks than visible GPUs (rehearsals): ranks share devices round-robin
        import torch
        ndev = max(1, torch.cuda.device_count())
        device = local % ndev
        if world > ndev and rank == 0:
            sys.stderr.write(f"bench: {world} ranks on {ndev} visible GPU(s): ranks share devices (rehearsal); "
                             "RCCL refuses two ranks on one device, so the fan-out legs report that error\n")
    B = a.batch
    # headline: the default (classic) parameters of configs[1]; the multi-bit blind rotation (same
    # client key, grouping 2) is measured beside it with the same protocol
    ck, ctx, cl = pbs_leg(a, "classic", dist, rank, world, device)
    ops, op_levels = (None, {}) if a.no_ops else ops_legs(ck, ctx, a.seed)
    if ops is not None and dist is not None:
        for k in ops:
            ops[k]["seconds"] = allmax(dist, ops[k]["seconds"])
        # every rank signs its own batch of 8 (config 5b): whole-job signatures per second
        b8 = ops["sign_fhe_with_k0_batch8_compat"]
        b8["signs_per_s"] = world * 8 / b8["seconds"]
    fan, fan_hung = None, False
    if world > 1 and not a.no_ops:
        fan, fan_hung = with_deadline(lambda: fanout_legs(ck, ctx, dist, rank, world, a.seed), FANOUT_DEADLINE_S)
        if fan_hung:
            fan = {"ranks": world, "error": f"fan-out legs exceeded {FANOUT_DEADLINE_S:.0f} s; abandoned"}
    mb = None
    if not a.no_multibit and not fan_hung:
        ck_mb, ctx_mb, mb = pbs_leg(a, "multibit", dist, rank, world, device)
        if not a.no_ops:
            mb_ops, _ = ops_legs(ck_mb, ctx_mb, a.seed)
            if dist is not None:
                for k in mb_ops:
                    mb_ops[k]["seconds"] = allmax(dist, mb_ops[k]["seconds"])
                mb_ops["sign_fhe_with_k0_batch8_compat"]["signs_per_s"] = (
                    world * 8 / mb_ops["sign_fhe_with_k0_batch8_compat"]["seconds"])
            mb["ops"] = mb_ops
            mb["biguint256_mul_seconds"] = mb_ops["biguint256_mul_compat"]["seconds"]
            mb["sign_fhe_with_k0_seconds"] = mb_ops["sign_fhe_with_k0_v0_compat"]["seconds"]
        ctx_mb.close()

    cpu = cpu_baseline(a.seed, a.cpu_seconds, op_levels) if rank == 0 and world == 1 and not a.no_cpu_baseline else None
    res, detail = compose_line(a, world, cl, ops, mb, fan, cpu)
    if rank == 0 and a.detail:
        try:
            os.makedirs(os.path.dirname(os.path.abspath(a.detail)), exist_ok=True)
            with open(a.detail, "w") as f:
                json.dump(detail, f, indent=1)
        except OSError as e:
            sys.stderr.write(f"bench: detail file not written: {e}\n")
    if rank == 0:
        print(json.dumps(res, separators=(",", ":")), file=out, flush=True)
    if fan_hung:  # a collective of the abandoned legs may still hold the stream: no orderly teardown
        abandon("fan-out legs hung")
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
