#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5t; mkdir -p $OUT
timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg --rounds 3 --warmup 1 --no-eval > $OUT/noeval.txt 2>&1 || { tail -20 $OUT/noeval.txt; exit 1; }
grep -E "^round" $OUT/noeval.txt; tail -1 $OUT/noeval.txt | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/cprof -o run -- python3 -u tools/bench_cifar.py --algorithm subavg --rounds 2 --warmup 1 --no-eval > $OUT/noeval_prof.txt 2>&1 || { tail -20 $OUT/noeval_prof.txt; exit 1; }
db=$(find /tmp/cprof -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" $OUT/noeval_kernels.txt --top 30 --window-ms 1400 > /dev/null 2>&1
head -20 $OUT/noeval_kernels.txt | cut -c1-140; grep TIMELINE $OUT/noeval_kernels.txt
