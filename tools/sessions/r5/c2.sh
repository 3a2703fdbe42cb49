#!/bin/bash
# A/B of the direct wgrad epilogue (1 = 1x1 layers only, 2 = every layer, 0 = off) on the CIFAR ResNet-18-GN benches
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5c2; mkdir -p $OUT
for alg in dispfl subavg; do
  for V in 0 1 2; do
    NIDT_WG_DIRECT=$V timeout -k 10 300 python -u tools/bench_cifar.py --algorithm $alg --rounds 2 --warmup 1 > $OUT/${alg}_$V.txt 2>&1 || { tail -20 $OUT/${alg}_$V.txt; exit 1; }
    echo "== $alg WG_DIRECT=$V $(tail -1 $OUT/${alg}_$V.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["s_round_each"])')"
  done
done
