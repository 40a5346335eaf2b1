"""Summarise a FHE_TRACE_LEVELS log (tools/level_trace.py stderr): levels, time and PBS per op,
bucketed by level size."""
import re, sys
cur = None; d = {}
for line in open(sys.argv[1]):
    if line.startswith("== ") and len(line.split()) == 2:
        cur = line.split()[1]; d[cur] = []
    m = re.match(r"\[level (\d+)\] (\d+) PBS ([\d.]+) ms", line)
    if m and cur:
        d[cur].append((int(m.group(2)), float(m.group(3))))
for k, v in d.items():
    print(k, len(v), "levels", round(sum(x[1] for x in v), 1), "ms", sum(x[0] for x in v), "PBS")
    b = {}
    for n, t in v:
        key = next(lim for lim in (128, 256, 512, 1024, 4096, 1 << 30) if n <= lim)
        c = b.setdefault(key, [0, 0.0, 0]); c[0] += 1; c[1] += t; c[2] += n
    for key in sorted(b):
        print(f"    <= {key:>10}: {b[key][0]:4d} levels {b[key][1]:8.1f} ms {b[key][2]:7d} PBS")
    if len(sys.argv) > 2 and k in sys.argv[2:]:
        print("   ", v)
