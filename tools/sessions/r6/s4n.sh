#!/bin/bash
# 16 / 32 / 64 clients per GPU (the 4- / 2- / 1-GPU per-rank loads of the strong-scaling bench): default (graphs on,
# no wgrad branch) vs eager steps with the wgrad branch, interleaved x2
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s4n; mkdir -p $OUT
for c in 16 32 64; do
  for rep in 1 2; do
    for arm in "1 0" "0 1"; do
      set -- $arm; g=$1; w=$2
      NIDT_HIP_GRAPHS=$g NIDT_AX_WGRAD_STREAM=$w timeout -k 10 300 python -u bench.py --clients $c --steps 10 --warmup 3 > $OUT/c${c}_g${g}_w${w}_$rep.txt 2>&1 || { tail -20 $OUT/c${c}_g${g}_w${w}_$rep.txt; exit 1; }
      echo "== clients $c rep $rep graphs=$g wgrad_stream=$w $(tail -1 $OUT/c${c}_g${g}_w${w}_$rep.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    done
  done
done
