#!/bin/bash
# CIFAR ResNet-18-GN (reference timed configs): current rounds/s of SubAvg / DisPFL + a kernel trace of each
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6z; mkdir -p $OUT
for alg in subavg dispfl; do
  timeout -k 10 400 python -u tools/bench_cifar.py --algorithm $alg --rounds 3 --warmup 1 > $OUT/${alg}.txt 2>&1 || { tail -20 $OUT/${alg}.txt; exit 1; }
  echo "== $alg $(tail -1 $OUT/${alg}.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["s_round_each"])')"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/cf_$alg -o run -- python3 -u tools/bench_cifar.py --algorithm $alg --rounds 2 --warmup 1 > $OUT/${alg}_prof.txt 2>&1 || { tail -20 $OUT/${alg}_prof.txt; exit 1; }
  db=$(find /tmp/cf_$alg -name "*.db" | head -1)
  steady=$(python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/${alg}_prof.txt') if l.startswith('{')][-1]
print(int(1000*sum(d['s_round_each'][1:])))")
  python3 tools/prof_summary.py "$db" $OUT/${alg}_kernels.txt --top 40 --window-ms "$steady" > /dev/null 2>&1
  head -25 $OUT/${alg}_kernels.txt | cut -c1-140
  grep -E "TOTAL|TIMELINE" $OUT/${alg}_kernels.txt
done
