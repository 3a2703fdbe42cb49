#!/bin/bash
# CIFAR DisPFL round phases (each bracketed by synchronize; tools/debug/round_phases.py)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s4i; mkdir -p $OUT
timeout -k 10 400 python3 -u tools/debug/round_phases.py --algorithm dispfl --rounds 2 --warmup 1 > $OUT/ph.txt 2>&1 || { tail -30 $OUT/ph.txt; exit 1; }
grep "^round" $OUT/ph.txt
