#!/bin/bash
# after the test-set fix: Tiny-ImageNet SubAvg at tiny.sh's batch 128, CIFAR SubAvg / DisPFL steady-round kernel traces
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s3m; mkdir -p $OUT
timeout -k 10 400 python -u tools/bench_cifar.py --dataset tiny --algorithm subavg --batch 128 --rounds 2 --warmup 1 > $OUT/tiny_subavg.txt 2>&1 || { tail -20 $OUT/tiny_subavg.txt; exit 1; }
echo "== tiny subavg b128 $(tail -1 $OUT/tiny_subavg.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["s_round_each"])')"
for alg in subavg dispfl; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/cf_$alg -o run -- python3 -u tools/bench_cifar.py --algorithm $alg --rounds 2 --warmup 1 > $OUT/${alg}_prof.txt 2>&1 || { tail -20 $OUT/${alg}_prof.txt; exit 1; }
  db=$(find /tmp/cf_$alg -name "*.db" | head -1)
  steady=$(python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/${alg}_prof.txt') if l.startswith('{')][-1]
print(int(1000*sum(d['s_round_each'][1:])))")
  python3 tools/prof_summary.py "$db" $OUT/${alg}_kernels.txt --top 40 --window-ms "$steady" > /dev/null 2>&1
  echo "== $alg"; grep -E "TOTAL|TIMELINE" $OUT/${alg}_kernels.txt
done
