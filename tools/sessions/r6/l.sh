#!/bin/bash
# sharded-path parity on one GPU: 64 clients as 1 rank with 8-client launches (--group 8) vs 8 gloo ranks of 8 clients
# (the headline's 8-GPU layout): per-client rows after one round's local training, and the global SNIP masks
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6l; mkdir -p $OUT
timeout -k 10 300 python -u bench.py --group 8 --steps 1 --warmup 0 --dump-rows /tmp/rows1 > $OUT/one.txt 2>&1 || { tail -20 $OUT/one.txt; exit 1; }
tail -1 $OUT/one.txt | cut -c1-160
NIDT_DIST_BACKEND=gloo timeout -k 20 400 python -u bench.py --gpus 8 --steps 1 --warmup 0 --dump-rows /tmp/rows8 > $OUT/eight.txt 2>&1 || { tail -30 $OUT/eight.txt; exit 1; }
grep "^{" $OUT/eight.txt | cut -c1-160
timeout -k 10 120 python -u tools/compare_rows.py /tmp/rows1 /tmp/rows8; echo "compare rc=$?"
timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --dump-rows /tmp/rows64 > $OUT/g64.txt 2>&1 || { tail -20 $OUT/g64.txt; exit 1; }
echo "== G=64 launches vs G=8 launches (one rank)"
timeout -k 10 120 python -u tools/compare_rows.py /tmp/rows64 /tmp/rows1; echo "compare rc=$?"
