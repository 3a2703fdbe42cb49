#!/bin/bash
# AlexNet3D 8 clients per GPU (the 8-GPU node's per-GPU load): weight gradients on a forked branch (NIDT_AX_WGRAD_STREAM)
# with captured hipGraph steps (default) and eager steps (NIDT_HIP_GRAPHS=0)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s3s; mkdir -p $OUT
for g in 1 0; do
  for w in 0 1; do
    NIDT_HIP_GRAPHS=$g NIDT_AX_WGRAD_STREAM=$w timeout -k 10 300 python -u bench.py --clients 8 --steps 20 --warmup 5 > $OUT/c8_g${g}_w$w.txt 2>&1 || { tail -20 $OUT/c8_g${g}_w$w.txt; exit 1; }
    echo "== c8 graphs=$g wgrad_stream=$w $(tail -1 $OUT/c8_g${g}_w$w.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
