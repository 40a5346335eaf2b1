#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh session into one JSON (committed under profiles/).

Per (kernel, grid size) and batch: mean counter value per dispatch.  HBM-side traffic per launch
follows MI355X_MICROARCH.md "HBM": FETCH_SIZE (KB) x 2 for 16-B/lane streaming reads on gfx950,
WRITE_SIZE (KB) as is; both count L2 memory-side requests, Infinity-Cache hits included.
Also copies the kernel-stats tables of the traced bench / ops runs.

usage: python3 tools/pmc_summary.py gpurun_out/prof_r1d profiles/r1/r1d_pmc_summary.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0]


def counters(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            key = f"{short(row['Kernel_Name'])} grid={row['Grid_Size']} wg={row['Workgroup_Size']}"
            acc[key][row["Counter_Name"]].append((row["Dispatch_Id"], float(row["Counter_Value"])))
    out = {}
    for k, cs in acc.items():
        out[k] = {}
        for c, vals in cs.items():
            per = defaultdict(float)
            for disp, v in vals:  # sum over dimensions within a dispatch, then mean over dispatches
                per[disp] += v
            out[k][c] = sum(per.values()) / len(per)
    return out


def stats(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            rows.append({"kernel": short(row["Name"]), "calls": int(row["Calls"]),
                         "total_ms": float(row["TotalDurationNs"]) / 1e6,
                         "avg_us": float(row["AverageNs"]) / 1e3, "pct": float(row["Percentage"])})
    return rows


def main():
    src, dst = sys.argv[1], sys.argv[2]
    res = {"source": os.path.basename(src.rstrip("/")), "kernel_stats": {}, "pmc": {}}
    for t in ("trace", "trace_ops"):
        if os.path.isdir(os.path.join(src, t)):
            res["kernel_stats"][t] = stats(os.path.join(src, t))
    merged = defaultdict(dict)
    for d in sorted(glob.glob(os.path.join(src, "pmc_*"))):
        if not os.path.isdir(d):
            continue
        batch = d.rsplit("_", 1)[-1]  # pmc_<B> or pmc_<kind>_<B> (kernels of both kinds differ by name)
        for k, cs in counters(d).items():
            merged[(batch, k)].update(cs)
    for (batch, k), cs in sorted(merged.items()):
        e = dict(cs)
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            e["hbm_side_bytes_per_launch"] = (2 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024
        if "TCC_HIT_sum" in e and "TCC_MISS_sum" in e:
            t = e["TCC_HIT_sum"] + e["TCC_MISS_sum"]
            e["l2_hit_rate"] = e["TCC_HIT_sum"] / t if t else None
        if "SQ_LDS_BANK_CONFLICT" in e and e.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_conflict_frac"] = e["SQ_LDS_BANK_CONFLICT"] / e["SQ_LDS_IDX_ACTIVE"]
        if e.get("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in e:
                    e[c + "_frac"] = e[c] / e["SQ_WAVE_CYCLES"]
        if "TA_TA_BUSY_sum" in e and e.get("GRBM_GUI_ACTIVE"):  # per CU (256) against per-XCD cycles (8)
            e["ta_busy_frac"] = (e["TA_TA_BUSY_sum"] / 256) / (e["GRBM_GUI_ACTIVE"] / 8)
        if e.get("SQ_WAVES"):
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU"):
                if c in e:
                    e[c + "_per_wave"] = e[c] / e["SQ_WAVES"]
        res["pmc"].setdefault(f"B={batch}", {})[k] = e
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps({b: {k: {c: v for c, v in e.items() if c.endswith(("frac", "rate", "launch", "per_wave"))}
                          for k, e in ks.items() if "blind" in k or "keyswitch" in k}
                      for b, ks in res["pmc"].items()}, indent=1))


if __name__ == "__main__":
    main()
