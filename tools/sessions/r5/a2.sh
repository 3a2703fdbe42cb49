#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5a2; mkdir -p $OUT
timeout -k 10 300 python -u tools/bench_conv2d.py > $OUT/conv2d.txt 2>&1 || { tail -20 $OUT/conv2d.txt; exit 1; }
cat $OUT/conv2d.txt
