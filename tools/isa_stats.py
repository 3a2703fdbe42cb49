"""Static instruction mix of the hot loop of each kernel in a gfx950 assembly file (``hipcc --cuda-device-only -S``).

For every kernel whose (demangled-ish) name matches the filter, finds the basic block with the most MFMA
instructions (the k-loop body after unrolling) and prints its counts per class: MFMA, VALU, SALU, LDS (ds_*),
VMEM (buffer_/global_), waitcnt, plus VALU/MFMA.  A static count, not a profile: the PMC ratios in
profiles/*pmc* are the measured counterpart.  Usage: ``python tools/isa_stats.py file.s [name-substring]``.
"""
from __future__ import annotations

import re
import sys
from collections import Counter


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def kernels(lines):
    cur, body = None, []
    for ln in lines:
        m = re.match(r"^(_Z\S+|k_\S+):\s*(;.*)?$", ln)
        if m:
            if cur:
                yield cur, body
            cur, body = m.group(1), []
            continue
        if cur and ln.startswith("\t.section") or (cur and ln.startswith(".Lfunc_end")):
            yield cur, body
            cur, body = None, []
            continue
        if cur:
            body.append(ln)
    if cur:
        yield cur, body


def blocks(body):
    blk, name = [], "entry"
    for ln in body:
        if re.match(r"^\.LBB\S+:", ln):
            yield name, blk
            name, blk = ln.split(":")[0], []
            continue
        s = ln.strip()
        if not s or s.startswith((";", ".")):
            continue
        blk.append(s.split()[0])
    yield name, blk


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    lines = open(path).read().splitlines()
    for k, body in kernels(lines):
        if filt not in k:
            continue
        best = max(blocks(body), key=lambda b: sum(1 for o in b[1] if o.startswith("v_mfma")))
        c = Counter(classify(o) for o in best[1])
        tot = Counter(classify(o) for _, b in blocks(body) for o in b)
        mf = max(1, c["mfma"])
        print("%-70s hot %-10s mfma %4d valu %4d salu %4d lds %3d vmem %3d wait %3d | valu/mfma %.2f salu/mfma %.2f"
              % (k[:70], best[0], c["mfma"], c["valu"], c["salu"], c["lds"], c["vmem"], c["wait"],
                 c["valu"] / mf, c["salu"] / mf))
        vc = Counter(o for o in best[1] if classify(o) == "valu")
        print("    top VALU:", ", ".join("%s %d" % kv for kv in vc.most_common(12)))
        print("    kernel total: mfma %d valu %d" % (tot["mfma"], tot["valu"]))


if __name__ == "__main__":
    main()
