"""Summarise a tools/gpu_l2ab.sh session: per build, the throughput kernel's L2 hit rate and L2 read
fills per launch (FETCH_SIZE x 2 KB on gfx950, MI355X_MICROARCH.md 'HBM'), beside the timing lines.
usage: python3 tools/l2ab_summary.py gpurun_out/TAG [kernel_substring]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "blind_rotate_qy"
ab = os.path.join(d, "sab", "ab.txt")
if os.path.exists(ab):
    print(open(ab).read().rstrip())
for pm in sorted(glob.glob(os.path.join(d, "pmc_*"))):
    if not os.path.isdir(pm):
        continue
    res = {}
    for f in glob.glob(os.path.join(pm, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kern in row["Kernel_Name"]:
                res.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    out = {k: sum(v) / len(v) for k, v in res.items()}
    if "TCC_HIT_sum" not in out or "FETCH_SIZE" not in out:
        continue
    hit, miss = out["TCC_HIT_sum"], out["TCC_MISS_sum"]
    print(f"{os.path.basename(pm)[4:]:12s} L2 hit {hit / (hit + miss):.3f}  L2 read fills "
          f"{out['FETCH_SIZE'] * 2 * 1024 / 1e9:.1f} GB per launch  GRBM_GUI_ACTIVE {out['GRBM_GUI_ACTIVE']:.0f}")
