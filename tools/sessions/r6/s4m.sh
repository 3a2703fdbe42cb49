#!/bin/bash
# 8 clients per GPU: default (graphs on, no wgrad branch) vs eager steps with the wgrad branch, interleaved x3
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s4m; mkdir -p $OUT
for rep in 1 2 3; do
  for arm in "1 0" "0 1" "1 1"; do
    set -- $arm; g=$1; w=$2
    NIDT_HIP_GRAPHS=$g NIDT_AX_WGRAD_STREAM=$w timeout -k 10 300 python -u bench.py --clients 8 --steps 30 --warmup 5 > $OUT/c8_g${g}_w${w}_$rep.txt 2>&1 || { tail -20 $OUT/c8_g${g}_w${w}_$rep.txt; exit 1; }
    echo "== rep $rep graphs=$g wgrad_stream=$w $(tail -1 $OUT/c8_g${g}_w${w}_$rep.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
