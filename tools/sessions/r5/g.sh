#!/bin/bash
# deferred metrics + pinned uploads: GPU suite, 64/8-client benches, kernel timeline of 8-client rounds
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5g; mkdir -p $OUT
true \


timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench64.txt 2>&1 || { tail -20 $OUT/bench64.txt; exit 1; }
tail -1 $OUT/bench64.txt
timeout -k 10 300 python -u bench.py --clients 8 --steps 30 --warmup 5 > $OUT/bench8.txt 2>&1 || { tail -20 $OUT/bench8.txt; exit 1; }
tail -1 $OUT/bench8.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof8 -o run -- python3 -u bench.py --clients 8 --steps 10 --warmup 3 > $OUT/prof8.txt 2>&1 || { tail -20 $OUT/prof8.txt; exit 1; }
DB=$(find /tmp/prof8 -name "*.db" | head -1)
python tools/prof_summary.py "$DB" $OUT/round_kernels_c8.txt --window-ms 550 --top 40 > /dev/null && tail -8 $OUT/round_kernels_c8.txt
