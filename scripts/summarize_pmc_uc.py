#!/usr/bin/env python
"""Summarise scripts/pmc_update_conv.sh: per (shape, tile, batch shape) the
per-dispatch averages of every counter of the conv kernel and the derived
ratios (MFMA busy share of the SIMD-cycles, wait shares of the wave-cycles,
VALU / SALU instructions per MFMA, LDS conflict share, L2 hit rate).

    python scripts/summarize_pmc_uc.py gpurun_out/pmc_uc
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

NSIMD = 256 * 4  # MI355X: 256 CUs x 4 SIMDs


def load(path):
    tot, disp = defaultdict(float), set()
    for r in csv.DictReader(open(path)):
        k = r.get("Kernel_Name", "")
        if "rs::conv::" not in k:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        disp.add(r.get("Dispatch_Id"))
    n = max(1, len(disp))
    return {k: v / n for k, v in tot.items()}, n


def main():
    d = sys.argv[1]
    cases = defaultdict(dict)
    us = {}
    for f in sorted(glob.glob(os.path.join(d, "*_p[0-9].csv"))):
        tag = os.path.basename(f)[:-7]
        c, _ = load(f)
        cases[tag].update(c)
        log = f[:-4] + ".log"
        if os.path.exists(log):
            m = re.search(r"tile\d+\s+([\d.]+)us\s+([\d.]+)TF", open(log).read())
            if m:
                us[tag] = (float(m.group(1)), float(m.group(2)))
    print("rocprofv3 --pmc, update-block convs at the tuned tiles (per dispatch; scripts/pmc_update_conv.sh)")
    print("mfma% = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs); wait% / active% of SQ_WAVE_CYCLES")
    for tag, c in cases.items():
        g = c.get("GRBM_GUI_ACTIVE", 0) / 8 or 1
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
        nm = mf / 16 if mf else 1  # 16x16x32 / 32x32x16 bf16: busy cycles per MFMA differ; report per-16-cycle unit
        t = us.get(tag, (0, 0))
        print(f"{tag}: {t[0]:.1f} us ({t[1]:.0f} TF/s graph-timed)")
        print(f"   mfma% {100 * mf / (g * NSIMD):5.1f}  active% {100 * c.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.1f}"
              f"  wait_any% {100 * c.get('SQ_WAIT_ANY', 0) / wc:5.1f}  wait_inst% {100 * c.get('SQ_WAIT_INST_ANY', 0) / wc:5.1f}"
              f"  waves {c.get('SQ_WAVES', 0):.0f}")
        print(f"   per 16 MFMA-busy cycles: VALU {c.get('SQ_INSTS_VALU', 0) / nm:5.2f}  SALU {c.get('SQ_INSTS_SALU', 0) / nm:5.2f}"
              f"  VMEM {c.get('SQ_INSTS_VMEM', 0) / nm:5.2f}  LDS {c.get('SQ_INSTS_LDS', 0) / nm:5.2f}"
              f"  SMEM {c.get('SQ_INSTS_SMEM', 0) / nm:5.2f}")
        lds = c.get("SQ_LDS_IDX_ACTIVE", 0) or 1
        hit, miss = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
        print(f"   lds_conflict% {100 * c.get('SQ_LDS_BANK_CONFLICT', 0) / lds:5.1f}  wait_inst_lds% "
              f"{100 * c.get('SQ_WAIT_INST_LDS', 0) / wc:5.1f}  L2 hit% {100 * hit / max(1, hit + miss):5.1f}"
              f"  TA_BUSY_avr {c.get('TA_BUSY_avr', 0):.3g}  GRBM/8 {g:.3g}")
        print("   raw: " + ", ".join(f"{k}={v:.4g}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
