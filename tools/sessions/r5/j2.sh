#!/bin/bash
# config 5 (3D ResNet-50, 256 clients): weight-gradient branch stream A/B (plain-reference branch)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5j2; mkdir -p $OUT
for V in 0 1; do
  NIDT_WGRAD_STREAM=$V timeout -k 10 500 python3 -u tools/config5_resnet3d.py --clients 256 --train-per-client 36 --test-per-client 9 --batch 4 --group 32 --rounds 3 --warmup 1 > $OUT/c5_$V.txt 2>&1 || { tail -20 $OUT/c5_$V.txt; exit 1; }
  echo "== WGRAD_STREAM=$V"; grep -E '^round' $OUT/c5_$V.txt; tail -1 $OUT/c5_$V.txt | cut -c1-200
done
