#!/bin/bash
# CIFAR SubAvg host profile (cProfile, eager steps) and the dispatch timeline of one replayed hipGraph step
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s3b; mkdir -p $OUT
timeout -k 10 300 python3 -u -m cProfile -o /tmp/sub.prof tools/bench_cifar.py --algorithm subavg --rounds 1 --warmup 1 > $OUT/subavg_cprof_run.txt 2>&1 || { tail -20 $OUT/subavg_cprof_run.txt; exit 1; }
python3 -c "
import pstats
p = pstats.Stats('/tmp/sub.prof'); p.sort_stats('tottime').print_stats(45)
p.sort_stats('cumulative').print_stats(60)" > $OUT/subavg_cprof.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/cfg -o run -- python3 -u tools/bench_cifar.py --algorithm subavg --rounds 1 --warmup 1 --graphs on > $OUT/subavg_graph_prof.txt 2>&1 || { tail -20 $OUT/subavg_graph_prof.txt; exit 1; }
db=$(find /tmp/cfg -name "*.db" | head -1)
python3 tools/step_timeline.py "$db" $OUT/subavg_graph_step.txt && tail -3 $OUT/subavg_graph_step.txt
