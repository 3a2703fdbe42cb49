#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5n; mkdir -p $OUT
timeout -k 10 300 python -u tools/bench_wgrad3d.py > $OUT/wg.txt 2>&1 || { tail -20 $OUT/wg.txt; exit 1; }
grep -v amdgpu.ids $OUT/wg.txt
