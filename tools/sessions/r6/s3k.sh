#!/bin/bash
# upper bound of removing the per-step dgrad-image transposes (k_pack_trans) from the CIFAR ResNet steps (probe)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s3k; mkdir -p $OUT
for alg in dispfl subavg; do
  for p in 0 1; do
    NIDT_PROBE_NOTRANS=$p timeout -k 10 400 python -u tools/debug/cifar_skip_ab.py --algorithm $alg --rounds 2 --warmup 1 > $OUT/${alg}_$p.txt 2>&1 || { tail -20 $OUT/${alg}_$p.txt; exit 1; }
    echo "== $alg notrans=$p $(tail -1 $OUT/${alg}_$p.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["s_round_each"])')"
  done
done
