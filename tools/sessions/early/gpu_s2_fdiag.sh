#!/bin/bash
# NOTE: NIDT_FWD_DIAG existed only in the temporary diagnostic build recorded in profiles/r2_ab_fwd_tri.txt (B-tile
# LDS-DMA skipped in the k-loop); on the tree this script just repeats the normal timings.
set -o pipefail
mkdir -p gpurun_out/fdiag; rm -f gpurun_out/fdiag/*
export PYTHONUNBUFFERED=1 KBENCH_EVAL=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for D in 0 1 2 3; do
  NIDT_FWD_DIAG=$D timeout -k 10 150 python tools/kbench.py 64 5 > gpurun_out/fdiag/kb64_d$D.txt 2>&1 || exit 1
done
grep -H "_fwd\|_dgrad" gpurun_out/fdiag/kb64_d*.txt | grep -v conv1
