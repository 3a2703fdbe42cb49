"""Summarise a rocprofv3 rocpd SQLite database (kernel-trace) into a per-kernel stats table.

``--window-ms W`` restricts the table to dispatches that start in the last W ms of the trace (the timed
rounds of a bench run come last) and adds a timeline line: wall span, GPU busy time (union of kernel
intervals), idle fraction and the largest inter-kernel gaps — the launch/sync overhead a hipGraph or
sync removal would recover.
"""
import argparse
import sqlite3


def main(db, top=30, out=None, window_ms=None):
    con = sqlite3.connect(db)
    cur = con.cursor()
    q = """select s.display_name, d.start, d.end
           from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id"""
    ev = cur.execute(q).fetchall()
    if window_ms:
        t_end = max(e for _, _, e in ev)
        ev = [x for x in ev if x[1] >= t_end - window_ms * 1e6]
    agg = {}
    for name, s, e in ev:
        a = agg.setdefault(name, [0, 0, 0])
        a[0] += 1
        a[1] += e - s
    rows = sorted(((n, a[0], a[1]) for n, a in agg.items()), key=lambda r: -r[2])
    tot = sum(r[2] for r in rows) or 1
    lines = ["%-90s %8s %12s %10s %6s" % ("kernel", "calls", "total_ms", "avg_us", "pct")]
    for name, n, s in rows[:top]:
        lines.append("%-90s %8d %12.3f %10.2f %6.2f" % (name[:90], n, s / 1e6, s / n / 1e3, 100.0 * s / tot))
    lines.append("TOTAL kernel time %.3f ms over %d kernels (%d dispatches)" % (tot / 1e6, len(rows), len(ev)))
    if ev:
        # the largest gaps with the kernels around them (host-side stalls show up as long gaps)
        sev = sorted(ev, key=lambda x: x[1])
        ctx, end_max, prev = [], sev[0][2], sev[0][0]
        for k in range(1, len(sev)):
            gap = sev[k][1] - end_max
            if gap > 0:
                ctx.append((gap, prev, sev[k][0], (sev[k][1] - sev[0][1]) / 1e6))
            if sev[k][2] > end_max:
                end_max, prev = sev[k][2], sev[k][0]
        ctx.sort(reverse=True)
        for gap, a, b, at in ctx[:6]:
            lines.append("GAP %.3f ms at +%.1f ms: after %s -> before %s" % (gap / 1e6, at, a[:70], b[:70]))
        iv = sorted((s, e) for _, s, e in ev)
        busy, gaps = 0, []
        cs, ce = iv[0]
        for s, e in iv[1:]:
            if s > ce:
                busy += ce - cs
                gaps.append(s - ce)
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        span = iv[-1][1] - iv[0][0]
        gaps.sort(reverse=True)
        lines.append("TIMELINE span %.3f ms, GPU busy %.3f ms, idle %.1f %%, %d gaps (sum %.3f ms; largest us: %s)"
                     % (span / 1e6, busy / 1e6, 100.0 * (span - busy) / max(span, 1), len(gaps), sum(gaps) / 1e6,
                        ", ".join("%.0f" % (g / 1e3) for g in gaps[:8])))
    txt = "\n".join(lines)
    print(txt)
    if out:
        open(out, "w").write(txt + "\n")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("out", nargs="?")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--window-ms", type=float, default=None)
    a = ap.parse_args()
    main(a.db, top=a.top, out=a.out, window_ms=a.window_ms)
