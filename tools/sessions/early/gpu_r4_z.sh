#!/bin/bash
# evaluation forms at 8 clients per GPU (the per-GPU load of the 8-GPU run), interleaved
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4z; mkdir -p $OUT
for arm in 1 0 1b 0b 1c 0c; do
  v=${arm%[bc]}
  NIDT_EVAL_STAGE=$v timeout -k 10 300 python bench.py --clients 8 --steps 30 --warmup 5 > $OUT/c8_s$arm.json 2>&1 || exit 1
  echo "c8 stage=$arm: $(grep -o '"value": [0-9.]*' $OUT/c8_s$arm.json)"
done
