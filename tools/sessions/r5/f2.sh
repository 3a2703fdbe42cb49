#!/bin/bash
# A/B: weight gradients on a branch stream (NIDT_WGRAD_STREAM=1) for the CIFAR ResNet-18-GN benches
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5f2; mkdir -p $OUT
for alg in subavg dispfl; do
  for V in 0 1; do
    NIDT_WGRAD_STREAM=$V timeout -k 10 300 python -u tools/bench_cifar.py --algorithm $alg --rounds 2 --warmup 1 > $OUT/${alg}_$V.txt 2>&1 || { tail -20 $OUT/${alg}_$V.txt; exit 1; }
    echo "== $alg WGRAD_STREAM=$V $(tail -1 $OUT/${alg}_$V.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["s_round_each"], d.get("last_round_metrics"))')"
  done
done
