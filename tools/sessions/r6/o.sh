#!/bin/bash
# 8-client step (the 8-GPU node's per-GPU load): small-grid tuning sweep over the existing A/B switches (kbench 8)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6o; mkdir -p $OUT
export KBENCH_EVAL=0
i=0
for cfg in "X=0" "NIDT_FWD_KSPLIT=2" "NIDT_FWD_KSPLIT=3" "NIDT_FWD_BP128=0" "NIDT_FWD_BP_THRESH=1024" "NIDT_FWD_NST=3" \
           "NIDT_WG_TRI_MINPOS=8192" "NIDT_WG_NSPLIT_FORCE=2" "NIDT_WG_NSPLIT_FORCE=6" "X=1"; do
  i=$((i+1))
  env $cfg timeout -k 10 120 python -u tools/kbench.py 8 > $OUT/k$i.txt 2>&1 || { tail -20 $OUT/k$i.txt; exit 1; }
  echo "== $cfg $(grep -o 'full train step [0-9.]* ms' $OUT/k$i.txt)"; grep -E "^conv[2345]_" $OUT/k$i.txt | awk '{printf "%s %s | ", $1, $2} END {print ""}'
done
