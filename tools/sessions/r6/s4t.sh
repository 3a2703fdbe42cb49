#!/bin/bash
# multi-rank rehearsal on ONE GPU with the [EAGER-BRANCH] defaults (ranks of <= 32 clients train in eager steps with
# the weight-gradient branch): 1 rank vs 2 and 8 gloo ranks sharing cuda:0, 64 clients (functional, not scaling)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s4t; mkdir -p $OUT
timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 > $OUT/one_rank.txt 2>&1 || { tail -20 $OUT/one_rank.txt; exit 1; }
tail -1 $OUT/one_rank.txt | cut -c1-900
NIDT_DIST_BACKEND=gloo timeout -k 20 300 python -u bench.py --gpus 2 --steps 2 --warmup 1 > $OUT/two_ranks.txt 2>&1 || { tail -30 $OUT/two_ranks.txt; exit 1; }
grep "^{" $OUT/two_ranks.txt | cut -c1-900
NIDT_DIST_BACKEND=gloo timeout -k 20 400 python -u bench.py --gpus 8 --steps 2 --warmup 1 > $OUT/eight_ranks.txt 2>&1 || { tail -30 $OUT/eight_ranks.txt; exit 1; }
grep "^{" $OUT/eight_ranks.txt | cut -c1-900
