#!/bin/bash
# [EAGER-BRANCH] follow-up: conv2 wgrad forked before (NIDT_WG2_EARLY=1) vs after the conv2 dgrad, 8 / 16 / 32 clients
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s4q; mkdir -p $OUT
for c in 8 16 32; do
  for rep in 1 2; do
    for e in 0 1; do
      NIDT_WG2_EARLY=$e timeout -k 10 300 python -u bench.py --clients $c --steps 10 --warmup 3 > $OUT/c${c}_e${e}_$rep.txt 2>&1 || { tail -20 $OUT/c${c}_e${e}_$rep.txt; exit 1; }
      echo "== clients $c rep $rep wg2_early=$e $(tail -1 $OUT/c${c}_e${e}_$rep.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    done
  done
done
