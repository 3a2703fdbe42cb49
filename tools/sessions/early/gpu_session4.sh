#!/bin/bash
# Re-verify on a fresh box after the container rebuild: GPU numerics tests, smoke, headline bench (64 clients),
# the per-GPU load of the 8-GPU run (8 clients on one GPU), and a kernel trace of the latter.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/bench64.txt 2>&1 || exit $?
timeout -k 10 200 python bench.py --clients 8 --steps 5 --warmup 1 --phase-timers > gpurun_out/bench8.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8 -o run -- python3 bench.py --clients 8 --steps 3 --warmup 1 > gpurun_out/prof8.txt 2>&1 || exit $?
