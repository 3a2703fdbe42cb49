#!/bin/bash
# conv1 wgrad mx: is the row loop bound by the staging loads' latency?  DBG=1 re-reads stage 0 every row (L2 hits)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5g; mkdir -p $OUT
for arm in 0 1 0 1; do
  NIDT_C1WG_DBG=$arm timeout -k 10 200 python -u tools/kbench.py 64 5 > $OUT/kb64_dbg$arm.txt 2>&1 || exit 1
  echo "dbg=$arm $(grep conv1_wgrad $OUT/kb64_dbg$arm.txt)"
done
