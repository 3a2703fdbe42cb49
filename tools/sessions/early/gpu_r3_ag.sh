#!/bin/bash
# CIFAR SubAvg round: kernel trace as CSV, summarised per (kernel, grid size) to see the small-grid conv costs
set -o pipefail
mkdir -p gpurun_out/r3ag
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/profag -o run -- python3 -u tools/bench_cifar.py \
  --algorithm subavg --rounds 1 --warmup 1 > gpurun_out/r3ag/run.txt 2>&1 || { tail -20 gpurun_out/r3ag/run.txt; exit 1; }
f=$(find /tmp/profag -name "*kernel_trace.csv" | head -1)
python3 - "$f" > gpurun_out/r3ag/grid_summary.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
t_end = max(int(r["End_Timestamp"]) for r in rows)
win = [r for r in rows if int(r["Start_Timestamp"]) >= t_end - 1.3e9]   # the timed round (~1.1 s)
agg = collections.defaultdict(lambda: [0, 0.0])
for r in win:
    k = (r["Kernel_Name"][:70], r.get("Grid_Size", r.get("Grid_Size_X", "?")), r.get("Workgroup_Size", r.get("Workgroup_Size_X", "?")))
    a = agg[k]; a[0] += 1; a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in agg.values())
print("window dispatches", len(win), "kernel us", round(tot))
print("%-72s %10s %6s %7s %10s %8s" % ("kernel", "grid", "wg", "calls", "total_us", "avg_us"))
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:70]:
    print("%-72s %10s %6s %7d %10.0f %8.1f" % (k[0], k[1], k[2], v[0], v[1], v[1] / v[0]))
print(list(rows[0].keys()))
PY
head -75 gpurun_out/r3ag/grid_summary.txt
