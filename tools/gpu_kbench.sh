#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/kbench.py 64 10 > gpurun_out/kbench64.txt 2>&1 || exit $?
timeout -k 10 200 python tools/kbench.py 8 10 > gpurun_out/kbench8.txt 2>&1 || exit $?
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
