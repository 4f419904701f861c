"""Summarise rocprofv3 --pmc counter CSVs per kernel (mean per dispatch) with the derived ratios used in DESIGN.md:
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs); wait / issue-stall / active shares
of SQ_WAVE_CYCLES; LDS bank-conflict share of SQ_LDS_IDX_ACTIVE.  usage: python tools/sq_summary.py <dir> [<dir>...]"""
import csv
import glob
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(\w+)(<[^()]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else name


def main(dirs):
    vals = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(path)):
                vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in sorted(vals.items()):
        if not any(x in k for x in ("mlp_kernel", "gemm_kernel", "window_attn", "rasterize", "subm")):
            continue
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        n = max(len(v) for v in cs.values())
        out = [f"{k[:64]:64s} n={n:4d}"]
        g = m.get("GRBM_GUI_ACTIVE")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and g:
            out.append(f"MFMA busy {100 * m['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * g / 8):5.1f}%")
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c, lab in (("SQ_WAIT_ANY", "wait"), ("SQ_WAIT_INST_ANY", "istall"), ("SQ_ACTIVE_INST_ANY", "active"),
                           ("SQ_WAIT_INST_LDS", "lds-stall")):
                if c in m:
                    out.append(f"{lab} {100 * m[c] / wc:5.1f}%")
        if m.get("SQ_LDS_IDX_ACTIVE"):
            out.append(f"LDS conflict {100 * m.get('SQ_LDS_BANK_CONFLICT', 0) / m['SQ_LDS_IDX_ACTIVE']:5.1f}%")
        if m.get("SQ_INSTS_MFMA"):
            out.append(f"VALU/MFMA {m.get('SQ_INSTS_VALU', 0) / m['SQ_INSTS_MFMA']:.2f}")
        if g:
            out.append(f"GRBM/8 {g / 8:9.0f} cyc")
        print("  ".join(out))


if __name__ == "__main__":
    main(sys.argv[1:])
