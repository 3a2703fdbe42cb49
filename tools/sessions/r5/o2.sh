#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5o2; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/bprof -o run -- python3 -u bench.py --steps 6 --warmup 2 > $OUT/bench_prof.txt 2>&1 || { tail -20 $OUT/bench_prof.txt; exit 1; }
db=$(find /tmp/bprof -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" $OUT/c64_kernels.txt --top 40 --window-ms 2400 > /dev/null 2>&1
head -30 $OUT/c64_kernels.txt | cut -c1-150; grep -E "TOTAL|TIMELINE" $OUT/c64_kernels.txt
for i in 1 2; do timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/b$i.txt 2>&1 || exit 1; tail -1 $OUT/b$i.txt | cut -c1-160; done
