#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5u2; mkdir -p $OUT
timeout -k 10 400 python -u tools/bench_cifar.py --dataset tiny --algorithm subavg --batch 128 --rounds 2 --warmup 1 > $OUT/tiny_subavg_b128.txt 2>&1 || { tail -20 $OUT/tiny_subavg_b128.txt; exit 1; }
tail -1 $OUT/tiny_subavg_b128.txt | cut -c1-300
