#!/bin/bash
# round-6 baseline: kbench at G=64 and G=8 with the default kernel set
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6a; mkdir -p $OUT
timeout -k 10 200 python -u tools/kbench.py 64 > $OUT/kb64.txt 2>&1 || { tail -20 $OUT/kb64.txt; exit 1; }
timeout -k 10 200 python -u tools/kbench.py 8 > $OUT/kb8.txt 2>&1 || { tail -20 $OUT/kb8.txt; exit 1; }
cat $OUT/kb64.txt $OUT/kb8.txt
