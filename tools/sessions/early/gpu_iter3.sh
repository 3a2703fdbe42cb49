#!/bin/bash
# Iteration check: conv/AlexNet numerics, kbench at 64 and 8 clients, 64-client bench.
set -o pipefail
mkdir -p gpurun_out/it3
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "${PYTEST_K:-conv3d or alexnet or graph or hip_conv or resnet}" > gpurun_out/it3/pytest.txt 2>&1 || exit $?
timeout -k 10 200 python tools/kbench.py 64 10 > gpurun_out/it3/kbench64.txt 2>&1 || exit $?
timeout -k 10 200 python tools/kbench.py 8 10 > gpurun_out/it3/kbench8.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/it3/bench64.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --clients 8 --steps 10 --warmup 3 > gpurun_out/it3/bench8.txt 2>&1 || exit $?
