#!/bin/bash
# A/B on one box: SubAvg first-epoch prune computed after training (NIDT_SUBAVG_LATE_PRUNE=1) vs between epochs
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5s2; mkdir -p $OUT
for V in 0 1 0 1; do
  NIDT_SUBAVG_LATE_PRUNE=$V timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg --rounds 3 --warmup 1 > $OUT/subavg_$V.txt 2>&1 || { tail -20 $OUT/subavg_$V.txt; exit 1; }
  echo "== LATE_PRUNE=$V $(tail -1 $OUT/subavg_$V.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["s_round_each"], d.get("last_round_metrics"))')"
done
