#!/bin/bash
# Headline bench + the 8-client per-GPU load, both with synchronised phase timers.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --phase-timers > gpurun_out/bench64.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 4 --warmup 1 > gpurun_out/bench64_nt.txt 2>&1 || exit $?
timeout -k 10 200 python bench.py --clients 8 --steps 10 --warmup 2 --phase-timers > gpurun_out/bench8.txt 2>&1 || exit $?
