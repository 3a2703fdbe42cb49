#!/bin/bash
# Small-grid forward/dgrad block shape: 64-position blocks below NIDT_FWD_BP_THRESH 256-position block-grids (default
# 256) vs 512 and 1024, at 8 clients.
set -o pipefail
mkdir -p gpurun_out/ab3
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "conv3d or alexnet" > gpurun_out/ab3/pytest.txt 2>&1 || exit $?
timeout -k 10 200 python tools/kbench.py 8 10 > gpurun_out/ab3/kbench8_256.txt 2>&1 || exit $?
NIDT_FWD_BP_THRESH=512 timeout -k 10 200 python tools/kbench.py 8 10 > gpurun_out/ab3/kbench8_512.txt 2>&1 || exit $?
NIDT_FWD_BP_THRESH=512 NIDT_FWD_NST=2 timeout -k 10 200 python tools/kbench.py 8 10 > gpurun_out/ab3/kbench8_512_nst2.txt 2>&1 || exit $?
