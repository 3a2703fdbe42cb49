#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5m; mkdir -p $OUT
timeout -k 10 300 python -u tools/bench_bnr.py > $OUT/bnr.txt 2>&1 || { tail -20 $OUT/bnr.txt; exit 1; }
grep -v amdgpu.ids $OUT/bnr.txt
