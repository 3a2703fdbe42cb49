#!/bin/bash
# Headline bench (1 GPU), 8-client per-GPU load of the 8-GPU run, and a rocprofv3 kernel profile of the bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench64.txt 2>&1 || exit $?
timeout -k 10 200 python bench.py --clients 8 --steps 10 --warmup 2 --phase-timers > gpurun_out/bench8.txt 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof64 -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof64.txt 2>&1 || exit $?
