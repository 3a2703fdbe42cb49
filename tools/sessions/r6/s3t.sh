#!/bin/bash
# CIFAR DisPFL (G = 100 lockstep steps): sweep of the existing small-grid / wgrad switches on the current tree
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s3t; mkdir -p $OUT
i=0
for e in X=0 NIDT_WG_DIRECT=2 NIDT_WG_DIRECT=0 NIDT_WGRAD_STREAM=0 NIDT_FWD_KSPLIT=1 NIDT_WG_NSPLIT_LEGACY=1 NIDT_WG_TRI=0 X=1; do
  i=$((i+1))
  env $e timeout -k 10 300 python -u tools/bench_cifar.py --algorithm dispfl --rounds 2 --warmup 1 > $OUT/d_$i.txt 2>&1 || { tail -20 $OUT/d_$i.txt; exit 1; }
  echo "== $e $(tail -1 $OUT/d_$i.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["s_round_each"])')"
done
