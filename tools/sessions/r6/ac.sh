#!/bin/bash
# CIFAR ResNet-18-GN SubAvg / DisPFL: eager steps (engine default) vs captured hipGraph steps, interleaved
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6ac; mkdir -p $OUT
for alg in subavg dispfl; do
  for gr in default on default on; do
    timeout -k 10 400 python -u tools/bench_cifar.py --algorithm $alg --rounds 3 --warmup 1 --graphs $gr > $OUT/${alg}_$gr.txt 2>&1 || { tail -20 $OUT/${alg}_$gr.txt; exit 1; }
    echo "== $alg graphs=$gr $(tail -1 $OUT/${alg}_$gr.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["s_round_each"], d["graph_stats"])')"
  done
done
