#!/usr/bin/env python3
"""Instruction census of a kernel's innermost loops from hipcc -S output (blocks LLVM annotates as
'Loop Header' / 'in Loop: Header=...').  Prints the largest loop: VALU count, LDS ops, barriers, and
the kernel descriptor's VGPR / AGPR / scratch / LDS.  Used to compare blind-rotate variants on CPU.
usage: python3 tools/loop_census.py file.s kernel_substring"""
import collections
import re
import sys


def census(path, kname):
    s = open(path).read()
    m = re.search(r"\.amdhsa_kernel (\S*%s\S*)\n(.*?)\.end_amdhsa_kernel" % re.escape(kname), s, re.S)
    d = dict(re.findall(r"\.amdhsa_(\w+) (\d+)", m.group(2)))
    sym = m.group(1)
    lines = s.split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    loops = collections.defaultdict(list)
    cur = None
    for l in lines[start:end]:
        t = l.strip()
        if re.match(r"^\.LBB\d+_\d+:", t):
            lab = t.split(":")[0][2:]  # ".LBB2_27" -> "BB2_27", the form of "Header=BB2_27"
            mh = re.search(r"Header=(BB\d+_\d+)", t)
            cur = lab if "Loop Header" in t else (mh.group(1) if mh else None)
            continue
        if cur and t and not t.startswith((".", ";")):
            loops[cur].append(t.split()[0])
    body = max(loops.values(), key=len)
    c = collections.Counter(body)
    valu = sum(n for k, n in c.items() if k.startswith("v_"))
    return {"vgpr": int(d["next_free_vgpr"]), "agpr_offset": int(d["accum_offset"]),
            "scratch": int(d["private_segment_fixed_size"]), "lds": int(d["group_segment_fixed_size"]),
            "loop_insts": len(body), "valu": valu, "f64": sum(n for k, n in c.items() if k.endswith("f64") or "_f64_" in k),
            "ds_read_b128": c["ds_read_b128"], "ds_write_b128": c["ds_write_b128"], "s_barrier": c["s_barrier"]}


if __name__ == "__main__":
    for f in sys.argv[1:-1]:
        print(f, census(f, sys.argv[-1]))
