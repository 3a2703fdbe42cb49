#!/bin/bash
# CIFAR SubAvg round phases (synchronised per phase)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s3e; mkdir -p $OUT
timeout -k 10 300 python3 -u tools/debug/round_phases.py --algorithm subavg --rounds 3 --warmup 1 > $OUT/phases.txt 2>&1 || { tail -20 $OUT/phases.txt; exit 1; }
grep "^round" $OUT/phases.txt
