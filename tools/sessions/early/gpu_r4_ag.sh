#!/bin/bash
# 8-client round kernel timeline and 64-client round kernel table after the k-step schedule changes
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4ag; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/c8prof -o run -- python3 bench.py --clients 8 --steps 20 \
  --warmup 3 > $OUT/bench_c8.json 2>&1 || { tail -5 $OUT/bench_c8.json; exit 1; }
grep '^{' $OUT/bench_c8.json | cut -c1-200
db=$(find /tmp/c8prof -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" $OUT/c8_round_kernels.txt --top 45 --window-ms 700 > /dev/null 2>&1
tail -3 $OUT/c8_round_kernels.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/c64prof -o run -- python3 bench.py --steps 4 \
  --warmup 2 > $OUT/bench_c64.json 2>&1 || { tail -5 $OUT/bench_c64.json; exit 1; }
grep '^{' $OUT/bench_c64.json | cut -c1-200
db=$(find /tmp/c64prof -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" $OUT/c64_round_kernels.txt --top 45 --window-ms 900 > /dev/null 2>&1
tail -3 $OUT/c64_round_kernels.txt
