#!/bin/bash
# Iteration check: AlexNet-path numerics tests, then the per-kernel bench at 8 and 64 clients and a profile of the
# 8-client bench (small-kernel costs).
set -o pipefail
mkdir -p gpurun_out/it2
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "${PYTEST_K:-conv1 or bn or alexnet or head or graph}" > gpurun_out/it2/pytest.txt 2>&1 || exit $?
timeout -k 10 200 python tools/kbench.py 8 10 > gpurun_out/it2/kbench8.txt 2>&1 || exit $?
timeout -k 10 200 python tools/kbench.py 64 10 > gpurun_out/it2/kbench64.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/it2/prof8 -o run -- python3 bench.py --clients 8 --steps 3 --warmup 1 > gpurun_out/it2/prof8.txt 2>&1 || exit $?
