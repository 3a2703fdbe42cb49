#!/bin/bash
# rocprofv3 kernel trace + stats of the bench, then the eager reference-semantics baseline.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof_bench.txt 2>&1 || exit $?
timeout -k 10 400 python3 tools/eager_baseline.py --clients 64 --rounds 1 > gpurun_out/eager_fp32.txt 2>&1
