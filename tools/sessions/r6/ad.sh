#!/bin/bash
# CIFAR SubAvg (10 clients per round, ResNet-18-GN): env sweep of the small-grid switches on the current tree
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6ad; mkdir -p $OUT
i=0
for cfg in "X=0" "NIDT_WGRAD_STREAM=0" "NIDT_WG_DIRECT=2" "NIDT_WG_NSPLIT_FORCE=1" "NIDT_FWD_KSPLIT=1" "NIDT_2D_SLAB=0" \
           "NIDT_2D_SLAB_BD=0" "NIDT_GN_HOLD=0" "NIDT_WG_DIRECT=0" "X=1"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg --rounds 3 --warmup 1 > $OUT/s$i.txt 2>&1 || { tail -20 $OUT/s$i.txt; exit 1; }
  echo "== $cfg $(tail -1 $OUT/s$i.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["s_round_each"])')"
done
