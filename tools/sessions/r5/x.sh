#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5x; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/dprof -o run -- python3 -u tools/bench_cifar.py --algorithm dispfl --rounds 1 --warmup 1 > $OUT/dispfl_prof.txt 2>&1 || { tail -20 $OUT/dispfl_prof.txt; exit 1; }
db=$(find /tmp/dprof -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" $OUT/dispfl_kernels.txt --top 40 --window-ms 3900 > /dev/null 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/sprof -o run -- python3 -u tools/bench_cifar.py --algorithm subavg --rounds 1 --warmup 1 > $OUT/subavg_prof.txt 2>&1 || { tail -20 $OUT/subavg_prof.txt; exit 1; }
db=$(find /tmp/sprof -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" $OUT/subavg_kernels.txt --top 40 --window-ms 770 > /dev/null 2>&1
head -30 $OUT/dispfl_kernels.txt | cut -c1-150; grep -E "TOTAL|TIMELINE" $OUT/dispfl_kernels.txt
head -30 $OUT/subavg_kernels.txt | cut -c1-150; grep -E "TOTAL|TIMELINE" $OUT/subavg_kernels.txt
