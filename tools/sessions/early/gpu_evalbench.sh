#!/bin/bash
# Eval-forward cost at the round's evaluation shape vs the training batch shape (tools/kbench.py eval line).
set -o pipefail
mkdir -p gpurun_out/ev
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 python tools/kbench.py 64 5 > gpurun_out/ev/kbench64.txt 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/ev/prof -o run -- python3 tools/kbench.py 64 3 > gpurun_out/ev/prof.txt 2>&1 || exit $?
find gpurun_out/ev/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/ev/kernel_stats.csv \; ; rm -rf gpurun_out/ev/prof
