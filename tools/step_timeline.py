"""Dispatch-by-dispatch timeline of ONE steady training step from a rocprofv3 kernel-trace database (rocpd SQLite).

Steps are delimited by a marker kernel that runs once per step (default: the image input stage ``k_img_input`` of
the 2-D engine; ``--marker k_conv1_fwd`` for AlexNet3D); only windows that contain the optimizer kernel
(``--must k_local_step``) count as training steps, and the median-length one is printed: start offset, duration,
the idle gap before it on its queue, queue, grid / workgroup size and the kernel name, plus per-queue busy time and
the launch count.  Used to find the critical path of the small lockstep steps (launch latency, side-stream joins).
Usage: ``python tools/step_timeline.py trace.db out.txt``.
"""
import argparse
import sqlite3


def main(db, out, marker, must, which):
    con = sqlite3.connect(db)
    cur = con.cursor()
    cols = [r[1] for r in cur.execute("pragma table_info(rocpd_kernel_dispatch)").fetchall()]
    qcol = "queue_id" if "queue_id" in cols else ("stream_id" if "stream_id" in cols else None)
    gx = "grid_size_x" if "grid_size_x" in cols else None
    wx = "workgroup_size_x" if "workgroup_size_x" in cols else None
    sel = ["s.display_name", "d.start", "d.end", ("d." + qcol) if qcol else "0",
           ("d." + gx) if gx else "0", ("d." + wx) if wx else "0"]
    ev = cur.execute("select %s from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id"
                     % ", ".join(sel)).fetchall()
    ev.sort(key=lambda x: x[1])
    marks = [i for i, e in enumerate(ev) if marker in e[0]]
    wins = []
    for a, b in zip(marks, marks[1:]):
        seg = ev[a:b]
        if any(must in e[0] for e in seg):
            wins.append((ev[b][1] - ev[a][1], a, b))
    if not wins:
        raise SystemExit("no step window (marker %r with %r inside); columns: %s" % (marker, must, cols))
    wins_sorted = sorted(wins)
    _, a, b = wins_sorted[len(wins_sorted) // 2] if which == "median" else wins[-2 if len(wins) > 1 else -1]
    seg = ev[a:b]
    t0 = seg[0][1]
    lines = ["# %d training-step windows; lengths us: min %.0f median %.0f max %.0f; columns: %s"
             % (len(wins), wins_sorted[0][0] / 1e3, wins_sorted[len(wins) // 2][0] / 1e3, wins_sorted[-1][0] / 1e3,
                ",".join(cols)),
             "%9s %8s %8s %6s %9s %5s  %s" % ("start_us", "dur_us", "gap_us", "queue", "grid", "wg", "kernel")]
    last_end = {}
    busy = {}
    for name, s, e, q, g, w in seg:
        gap = (s - last_end[q]) / 1e3 if q in last_end else 0.0
        last_end[q] = max(last_end.get(q, 0), e)
        busy[q] = busy.get(q, 0) + (e - s)
        lines.append("%9.1f %8.1f %8.1f %6s %9s %5s  %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, q, g, w, name[:110]))
    span = (seg[-1][2] - t0) / 1e3
    lines.append("STEP span %.1f us, %d dispatches; busy per queue (us): %s" % (
        (ev[b][1] - t0) / 1e3, len(seg), ", ".join("%s: %.1f" % (q, v / 1e3) for q, v in sorted(busy.items()))))
    lines.append("last kernel end at %.1f us" % span)
    # where the rest of the trace's time goes: the step windows' total against the whole span, and the longest
    # windows (epoch boundaries, partial batches, evaluation) with the kernels that fill them
    tot = (ev[-1][2] - ev[0][1]) / 1e3
    lines.append("TRACE span %.1f ms; %d step windows sum %.1f ms (median %.0f us)" % (
        tot / 1e3, len(wins), sum(w[0] for w in wins) / 1e6, wins_sorted[len(wins) // 2][0] / 1e3))
    for ln, a2, b2 in sorted(wins, reverse=True)[:8]:
        agg = {}
        for name, s, e, *_ in ev[a2:b2]:
            agg[name] = agg.get(name, 0) + (e - s)
        top = sorted(agg.items(), key=lambda kv: -kv[1])[:4]
        lines.append("  window %.1f us at +%.1f ms, %d dispatches: %s" % (
            ln / 1e3, (ev[a2][1] - ev[0][1]) / 1e6, b2 - a2,
            "; ".join("%s %.0f us" % (n.split("(")[0][-48:], v / 1e3) for n, v in top)))
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("out")
    ap.add_argument("--marker", default="k_img_input")
    ap.add_argument("--must", default="k_local_step")
    ap.add_argument("--which", default="median", choices=["median", "last"])
    a = ap.parse_args()
    main(a.db, a.out, a.marker, a.must, a.which)
