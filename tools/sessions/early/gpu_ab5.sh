#!/bin/bash
# 128-position forward blocks for one-block-per-CU grids (conv3-5 at 8 clients) vs NIDT_FWD_BP128=0.
set -o pipefail
mkdir -p gpurun_out/ab5
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "conv3d or alexnet or graph" > gpurun_out/ab5/pytest.txt 2>&1 || exit $?
KBENCH_EVAL=0 timeout -k 10 200 python tools/kbench.py 8 10 > gpurun_out/ab5/kbench8_new.txt 2>&1 || exit $?
NIDT_FWD_BP128=0 KBENCH_EVAL=0 timeout -k 10 200 python tools/kbench.py 8 10 > gpurun_out/ab5/kbench8_old.txt 2>&1 || exit $?
KBENCH_EVAL=0 timeout -k 10 200 python tools/kbench.py 8 10 > gpurun_out/ab5/kbench8_new2.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --clients 8 --steps 10 --warmup 3 > gpurun_out/ab5/bench8_new.txt 2>&1 || exit $?
NIDT_FWD_BP128=0 timeout -k 10 300 python bench.py --clients 8 --steps 10 --warmup 3 > gpurun_out/ab5/bench8_old.txt 2>&1 || exit $?
