#!/bin/bash
# diagnostic: conv2 slab kernels with the per-kd union reloads skipped (timing only)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5s; mkdir -p $OUT
export KBENCH_EVAL=0
for V in 0 1 0 1; do
  NIDT_SLAB_DBG=$V timeout -k 10 200 python -u tools/kbench.py 64 > $OUT/kb_$V.txt 2>&1 || { tail -20 $OUT/kb_$V.txt; exit 1; }
  echo "== DBG=$V"; grep -E "full train step|conv2" $OUT/kb_$V.txt
done
