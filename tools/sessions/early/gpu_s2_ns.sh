#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/ns; rm -f gpurun_out/ns/*
export PYTHONUNBUFFERED=1 KBENCH_EVAL=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for F in 10 12 14 16 20; do
  if [ $F = 0 ]; then timeout -k 10 150 python tools/kbench.py 64 10 > gpurun_out/ns/kb_$F.txt 2>&1 || exit 1
  else NIDT_WG_NSPLIT_FORCE=$F timeout -k 10 150 python tools/kbench.py 64 10 > gpurun_out/ns/kb_$F.txt 2>&1 || exit 1; fi
done
grep -H "conv2_wgrad" gpurun_out/ns/kb_*.txt
