#!/bin/bash
# Split-K forward/dgrad for small grids: numerics, then kbench / bench at 8 clients with the default rule and with
# NIDT_FWD_KSPLIT=1 (no split), and the 64-client kbench (unchanged path).
set -o pipefail
mkdir -p gpurun_out/ab4
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "splitk or conv3d or alexnet or graph" > gpurun_out/ab4/pytest.txt 2>&1 || exit $?
timeout -k 10 200 python tools/kbench.py 8 10 > gpurun_out/ab4/kbench8_new.txt 2>&1 || exit $?
NIDT_FWD_KSPLIT=1 timeout -k 10 200 python tools/kbench.py 8 10 > gpurun_out/ab4/kbench8_old.txt 2>&1 || exit $?
timeout -k 10 200 python tools/kbench.py 32 10 > gpurun_out/ab4/kbench32_new.txt 2>&1 || exit $?
NIDT_FWD_KSPLIT=1 timeout -k 10 200 python tools/kbench.py 32 10 > gpurun_out/ab4/kbench32_old.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --clients 8 --steps 10 --warmup 3 > gpurun_out/ab4/bench8_new.txt 2>&1 || exit $?
NIDT_FWD_KSPLIT=1 timeout -k 10 300 python bench.py --clients 8 --steps 10 --warmup 3 > gpurun_out/ab4/bench8_old.txt 2>&1 || exit $?
