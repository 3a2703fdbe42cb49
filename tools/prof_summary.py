"""Summarise a rocprofv3 rocpd SQLite database (kernel-trace) into a per-kernel stats table."""
import sqlite3
import sys


def main(db, top=30, out=None):
    con = sqlite3.connect(db)
    cur = con.cursor()
    cols = [r[1] for r in cur.execute("pragma table_info(rocpd_kernel_dispatch)")]
    q = """select s.display_name, count(*), sum(d.end - d.start), avg(d.end - d.start), min(d.end-d.start), max(d.end-d.start)
           from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
           group by s.display_name order by sum(d.end - d.start) desc"""
    rows = cur.execute(q).fetchall()
    tot = sum(r[2] for r in rows)
    lines = ["%-90s %8s %12s %10s %6s" % ("kernel", "calls", "total_ms", "avg_us", "pct")]
    for name, n, s, a, mn, mx in rows[:top]:
        lines.append("%-90s %8d %12.3f %10.2f %6.2f" % (name[:90], n, s / 1e6, a / 1e3, 100.0 * s / tot))
    lines.append("TOTAL kernel time %.3f ms over %d kernels (%d dispatches)" % (tot / 1e6, len(rows), sum(r[1] for r in rows)))
    txt = "\n".join(lines)
    print(txt)
    if out:
        open(out, "w").write(txt + "\n")


if __name__ == "__main__":
    main(sys.argv[1], out=sys.argv[2] if len(sys.argv) > 2 else None)
