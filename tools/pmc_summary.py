"""Summarise rocprofv3 ``--pmc`` CSV passes (gpurun_out/pmc/p*/.../*counter_collection.csv) into one table:
mean counter value per dispatch for each kernel, plus derived ratios (MFMA busy %, VALU/MFMA instruction
mix, LDS bank-conflict %, issue-stall %).  Usage: python tools/pmc_summary.py gpurun_out/pmc [out.txt]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(root):
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per-dispatch values]
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        names = {}
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
                did = row.get("Dispatch_Id") or row.get("Correlation_Id")
                c = row.get("Counter_Name")
                per[(did, c)] += float(row.get("Counter_Value") or 0)
                names[did] = k
        for (did, c), v in per.items():
            vals[names[did]][c].append(v)
    return vals


def short(k):
    k = k.replace("nidt::", "")
    return k.split("(")[0][:48]


def main(root, out=None):
    vals = load(root)
    lines = []
    for k in sorted(vals, key=lambda x: short(x)):
        c = {n: sum(v) / len(v) for n, v in vals[k].items()}
        lines.append("== %s  (%d dispatches)" % (short(k), max(len(v) for v in vals[k].values())))
        for n in sorted(c):
            lines.append("   %-26s %16.0f" % (n, c[n]))
        d = []
        if c.get("SQ_BUSY_CYCLES") and c.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            # SQ_VALU_MFMA_BUSY_CYCLES is summed over SIMDs; SQ_BUSY_CYCLES over SEs (quad-cycles per SE)
            d.append("mfma_busy_per_simd_cycles=%.0f" % (c["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024))
            if c.get("GRBM_GUI_ACTIVE"):
                # MFMA pipe busy fraction: busy cycles over 1024 SIMDs x elapsed cycles (GRBM_GUI_ACTIVE sums 8 XCDs)
                d.append("MFMA_busy=%.1f%%" % (100.0 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * c["GRBM_GUI_ACTIVE"] / 8)))
        if c.get("SQ_INSTS_MFMA"):
            d.append("valu/mfma=%.2f lds/mfma=%.2f" % (c.get("SQ_INSTS_VALU", 0) / c["SQ_INSTS_MFMA"],
                                                      c.get("SQ_INSTS_LDS", 0) / c["SQ_INSTS_MFMA"]))
        if c.get("SQ_LDS_IDX_ACTIVE"):
            d.append("lds_conflict=%.1f%%" % (100.0 * c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"]))
        if c.get("SQ_WAVE_CYCLES"):
            d.append("wait_inst=%.1f%% wait_any=%.1f%% active=%.1f%%" % (
                100.0 * c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"],
                100.0 * c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"],
                100.0 * c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]))
        if d:
            lines.append("   derived: " + "; ".join(d))
    txt = "\n".join(lines)
    print(txt)
    if out:
        open(out, "w").write(txt + "\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
