#!/bin/bash
# CIFAR SubAvg / DisPFL after the per-client test-set size fix (reference: ~100 test samples per client)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s3g; mkdir -p $OUT
for alg in subavg dispfl; do
  timeout -k 10 400 python -u tools/bench_cifar.py --algorithm $alg --rounds 3 --warmup 1 > $OUT/${alg}.txt 2>&1 || { tail -20 $OUT/${alg}.txt; exit 1; }
  echo "== $alg $(tail -1 $OUT/${alg}.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["s_round_each"])')"
done
timeout -k 10 300 python3 -u tools/debug/round_phases.py --algorithm subavg --rounds 2 --warmup 1 > $OUT/phases.txt 2>&1 || { tail -20 $OUT/phases.txt; exit 1; }
grep "^round" $OUT/phases.txt
