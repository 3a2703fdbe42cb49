#!/bin/bash
# CIFAR SubAvg: per-launch times of the grouped test evaluation
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s3f; mkdir -p $OUT
timeout -k 10 300 python3 -u tools/debug/eval_launches.py --algorithm subavg --rounds 2 --warmup 1 > $OUT/eval.txt 2>&1 || { tail -20 $OUT/eval.txt; exit 1; }
grep -A 60 "^eval_grouped" $OUT/eval.txt | head -80
