#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5v2; mkdir -p $OUT
timeout -k 10 400 python -u -m cProfile -o /tmp/sa.prof tools/bench_cifar.py --algorithm subavg --rounds 3 --warmup 1 --no-eval > $OUT/run.txt 2>&1 || { tail -20 $OUT/run.txt; exit 1; }
grep -E "^round" $OUT/run.txt
python3 -c "
import pstats
p = pstats.Stats('/tmp/sa.prof')
p.sort_stats('tottime').print_stats(45)
" > $OUT/prof_tottime.txt 2>&1
python3 -c "
import pstats
p = pstats.Stats('/tmp/sa.prof')
p.sort_stats('cumulative').print_stats(60)
" > $OUT/prof_cum.txt 2>&1
head -70 $OUT/prof_tottime.txt | tail -45
