#!/usr/bin/env python3
"""Short per-kernel readout of a tools/pmc_passes.sh directory: instructions per wave, issue
utilisation and stall fractions (MI355X_MICROARCH.md counter meanings; GRBM_GUI_ACTIVE summed over
the 8 XCDs).  usage: python3 tools/pmc_brief.py gpurun_out/DIR [kernel-substring]"""
import sys
sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import counters  # noqa: E402

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "blind_rotate"
for k, v in counters(d).items():
    if pat not in k:
        continue
    w = v.get("SQ_WAVES", 1.0)
    cyc = v.get("GRBM_GUI_ACTIVE", 0.0) / 8  # per XCD
    print(k)
    print(f"  XCD cycles {cyc:.4g}")
    for n in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU"):
        if n in v:
            print(f"  {n}/wave {v[n] / w:.5g}")
    if "SQ_INSTS_VALU" in v and cyc:
        print(f"  VALU issue utilisation (4 cycles/instr, 1024 SIMDs) {v['SQ_INSTS_VALU'] * 4 / (1024 * cyc):.3f}")
    wc = v.get("SQ_WAVE_CYCLES")
    if wc:
        for n in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_WAIT_ANY",
                  "SQ_ACTIVE_INST_LDS"):
            if n in v:
                print(f"  {n}/WAVE_CYCLES {v[n] / wc:.3f}")
    if "SQ_LDS_BANK_CONFLICT" in v:
        print(f"  LDS bank-conflict cycles/wave {v['SQ_LDS_BANK_CONFLICT'] / w:.4g}")
    if "TA_TA_BUSY_sum" in v and cyc:
        print(f"  TA busy {v['TA_TA_BUSY_sum'] / (256 * cyc):.3f}")
