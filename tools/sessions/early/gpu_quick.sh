#!/bin/bash
# Quick kernel iteration on the GPU box: conv/alexnet numerics tests, then the per-kernel microbench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 420 python -m pytest tests/test_gpu_kernels.py -q -x -m gpu ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_quick.txt 2>&1 || exit $?
timeout -k 10 300 python tools/kbench.py 64 10 > gpurun_out/kbench64.txt 2>&1 || exit $?
