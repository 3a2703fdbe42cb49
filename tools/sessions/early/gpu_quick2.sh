#!/bin/bash
# Kernel iteration: numerics tests of the AlexNet path, then the per-kernel microbench at G=64 and G=8.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "${PYTEST_K:-conv1 or alexnet}" > gpurun_out/pytest_quick.txt 2>&1 || exit $?
timeout -k 10 200 python tools/kbench.py 64 10 > gpurun_out/kbench64.txt 2>&1 || exit $?
timeout -k 10 200 python tools/kbench.py 8 10 > gpurun_out/kbench8.txt 2>&1 || exit $?
