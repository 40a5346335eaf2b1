"""Level sizes and synchronised level times of one op (FHE_DEBUG=levels set by the caller): compat / fast
256-bit BigUintFHE mul, or the 256-bit / encrypted division; a summary by level-size class at the end.
usage: FHE_DEBUG=levels python3 tools/op_levels.py compat|fast|div"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if os.environ.get("OP_LEVELS_CHILD") != "1":  # run the op in a child, parse its stderr
    r = subprocess.run([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], capture_output=True, text=True,
                       env=dict(os.environ, OP_LEVELS_CHILD="1", FHE_DEBUG="levels"), timeout=600)
    sys.stdout.write(r.stdout)
    lv = [(int(m.group(1)), float(m.group(2))) for m in re.finditer(r"\[level \d+\] (\d+) PBS ([\d.]+) ms", r.stderr)]
    marks = [i for i, l in enumerate(r.stderr.splitlines()) if l.startswith("=== timed")]
    lines = r.stderr.splitlines()
    timed = [(int(m.group(1)), float(m.group(2))) for l in lines[marks[0]:] if (m := re.search(r"\[level \d+\] (\d+) PBS ([\d.]+) ms", l))] if marks else lv
    cls = {"<=256": (0, 256), "257-3071": (257, 3071), ">=3072": (3072, 1 << 30)}
    print(f"levels {len(timed)}, PBS {sum(g for g, _ in timed)}, synchronised level time {sum(t for _, t in timed):.1f} ms")
    for k, (lo, hi) in cls.items():
        sel = [(g, t) for g, t in timed if lo <= g <= hi]
        print(f"  {k:9s}: {len(sel):4d} levels, {sum(g for g, _ in sel):7d} PBS, {sum(t for _, t in sel):8.1f} ms")
    sys.exit(r.returncode)

sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
import json  # noqa: E402
import time  # noqa: E402

from fhe_sign import COMPAT, FAST, BigUintFHE, Context, FheUint256, generate_keys, set_server_key  # noqa: E402

op = sys.argv[1]
ck, sk = generate_keys(seed=0x5167)
ctx = Context(0)
ctx.set_server_key(sk)
set_server_key(ctx)
g = json.load(open(os.path.join(ROOT, "tests", "golden", "biguint_vectors.json")))["mul"][0]
val = lambda limbs: sum(int(x) << (32 * i) for i, x in enumerate(limbs))  # noqa: E731
a, b = val(g["a"]), val(g["b"])
if op in ("compat", "fast"):
    A, B = BigUintFHE.new(a, ck), BigUintFHE.new(b, ck)
    fn = lambda: A.mul(B, COMPAT if op == "compat" else FAST)  # noqa: E731
    check = (lambda r: r.decrypt_limbs(ck) == [int(x) for x in g["out"]]) if op == "compat" else (lambda r: r.to_biguint(ck) == a * b)
else:
    d = (1 << 127) | 12345
    A, D = FheUint256.try_encrypt(a, ck), FheUint256.try_encrypt(d, ck)
    fn = lambda: A.div_rem(D)  # noqa: E731
    check = lambda r: (r[0].decrypt(ck), r[1].decrypt(ck)) == (a // d, a % d)  # noqa: E731
assert check(fn())
print("=== timed", file=sys.stderr, flush=True)
t0 = time.perf_counter()
r = fn()
ok = check(r)
print(f"{op}: {time.perf_counter() - t0:.3f} s with every level synchronised, ok={ok}", flush=True)
ctx.close()
