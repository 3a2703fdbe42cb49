#!/bin/bash
# wgrad slab kernel with the asm-issued stage DMA ([ADMA]) vs the tri kernel (kbench 64 / 8), + slab wgrad numerics
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6ab; mkdir -p $OUT
NIDT_WG_SLAB=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad" > $OUT/t.txt 2>&1 || { grep -E "Error|assert|FAILED|passed|failed" $OUT/t.txt | tail -20; exit 1; }
tail -1 $OUT/t.txt
export KBENCH_EVAL=0
i=0
for G in 64 8; do
for cfg in "X=0" "NIDT_WG_SLAB=1" "NIDT_WG_SLAB=1 NIDT_WGS_ADMA=0" "X=1"; do
  i=$((i+1))
  env $cfg timeout -k 10 150 python -u tools/kbench.py $G > $OUT/k$i.txt 2>&1 || { tail -20 $OUT/k$i.txt; exit 1; }
  echo "== G=$G $cfg $(grep -o 'full train step [0-9.]* ms' $OUT/k$i.txt)"; grep -E "^conv[2345]_wgrad" $OUT/k$i.txt | awk '{printf "%s %s | ", $1, $2} END {print ""}'
done
done
