#!/bin/bash
# Pipeline depth for the 128-position small-grid blocks: NIDT_FWD_NST=3 (all forward convs) vs default, 8 clients.
set -o pipefail
mkdir -p gpurun_out/ab6
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NIDT_FWD_NST=3 KBENCH_EVAL=0 timeout -k 10 200 python tools/kbench.py 8 10 > gpurun_out/ab6/kbench8_nst3.txt 2>&1 || exit $?
KBENCH_EVAL=0 timeout -k 10 200 python tools/kbench.py 8 10 > gpurun_out/ab6/kbench8_def.txt 2>&1 || exit $?
