#!/bin/bash
# GroupNorm backward: hold the bf16 dy in registers for more rows (NIDT_GN_HOLD) now that no mask is held
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s3p; mkdir -p $OUT
for alg in dispfl subavg; do
  for h in 4 8 16; do
    NIDT_GN_HOLD=$h timeout -k 10 400 python -u tools/bench_cifar.py --algorithm $alg --rounds 3 --warmup 1 > $OUT/${alg}_$h.txt 2>&1 || { tail -20 $OUT/${alg}_$h.txt; exit 1; }
    echo "== $alg gn_hold=$h $(tail -1 $OUT/${alg}_$h.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["s_round_each"])')"
  done
done
