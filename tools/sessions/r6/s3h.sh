#!/bin/bash
# CIFAR DisPFL (G = 100 lockstep steps): kernel stats of the steady round and one step's dispatch timeline
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s3h; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/dp -o run -- python3 -u tools/bench_cifar.py --algorithm dispfl --rounds 1 --warmup 1 > $OUT/prof.txt 2>&1 || { tail -20 $OUT/prof.txt; exit 1; }
db=$(find /tmp/dp -name "*.db" | head -1)
steady=$(python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/prof.txt') if l.startswith('{')][-1]
print(int(1000*sum(d['s_round_each'])))")
python3 tools/prof_summary.py "$db" $OUT/kernels.txt --top 45 --window-ms "$steady" > /dev/null
python3 tools/step_timeline.py "$db" $OUT/step.txt
head -30 $OUT/kernels.txt | cut -c1-150; grep -E "TIMELINE" $OUT/kernels.txt; tail -12 $OUT/step.txt | cut -c1-250
