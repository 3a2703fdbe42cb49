#!/bin/bash
# timing diagnostic of the small-grid conv kernels (CIFAR SubAvg round): per (kernel, grid) durations with the full
# k-loop, without k-steps (launch + prologue + epilogue) and without MFMAs (loads + LDS reads + barriers)
set -o pipefail
mkdir -p gpurun_out/r3ar
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for d in 3 4; do
  export NIDT_FWD_DIAG=$d
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/profar$d -o run -- python3 -u tools/bench_cifar.py \
    --algorithm subavg --rounds 1 --warmup 1 > gpurun_out/r3ar/run$d.txt 2>&1
  echo "diag $d rc=$?"
  f=$(find /tmp/profar$d -name "*kernel_trace.csv" | head -1)
  [ -n "$f" ] || exit 1
  python3 - "$f" > gpurun_out/r3ar/grid$d.txt <<'PY'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_conv_fwd_dma" in r["Kernel_Name"]]
t_end = max(int(r["End_Timestamp"]) for r in rows)
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    if int(r["Start_Timestamp"]) < t_end - 1.3e9:
        continue
    k = (r["Kernel_Name"].split("(")[0][-40:], r["Grid_Size_X"], r["Workgroup_Size_X"])
    a = agg[k]; a[0] += 1; a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:16]:
    print("%-42s %8s %5s %6d %9.0f %7.1f" % (k[0], k[1], k[2], v[0], v[1], v[1] / v[0]))
PY
  cat gpurun_out/r3ar/grid$d.txt
done
