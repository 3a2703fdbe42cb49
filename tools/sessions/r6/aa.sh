#!/bin/bash
# 64-client step: sweep of the existing A/B switches since the round-6 kernel changes ([ADMA] etc.) (kbench 64)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6aa; mkdir -p $OUT
export KBENCH_EVAL=0
i=0
for cfg in "X=0" "NIDT_WG_SLAB=1" "NIDT_WG_TRI_NCH=2" "NIDT_WG_NCH=2" "NIDT_FWD_VOL=1" "NIDT_WG_NSPLIT_FORCE=2" \
           "NIDT_WG_NSPLIT_FORCE=4" "NIDT_SLAB_NA=3" "NIDT_AX_WGRAD_STREAM=0" "NIDT_WG2_EARLY=1" "X=1"; do
  i=$((i+1))
  env $cfg timeout -k 10 150 python -u tools/kbench.py 64 > $OUT/k$i.txt 2>&1 || { tail -20 $OUT/k$i.txt; exit 1; }
  echo "== $cfg $(grep -o 'full train step [0-9.]* ms' $OUT/k$i.txt)"; grep -E "^conv[2345]_" $OUT/k$i.txt | awk '{printf "%s %s | ", $1, $2} END {print ""}'
done
