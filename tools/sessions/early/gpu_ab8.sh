#!/bin/bash
# 512-position forward/dgrad blocks on large grids (NIDT_FWD_BP512=1) vs 256: numerics with the variant on, then
# kbench and bench at 64 clients both ways.
set -o pipefail
mkdir -p gpurun_out/ab8
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NIDT_FWD_BP512=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "conv3d_fwd_stats or conv3d_wgrad or alexnet or graph" > gpurun_out/ab8/pytest.txt 2>&1 || exit $?
NIDT_FWD_BP512=1 KBENCH_EVAL=0 timeout -k 10 200 python tools/kbench.py 64 8 > gpurun_out/ab8/kbench64_bp512.txt 2>&1 || exit $?
KBENCH_EVAL=0 timeout -k 10 200 python tools/kbench.py 64 8 > gpurun_out/ab8/kbench64_def.txt 2>&1 || exit $?
NIDT_FWD_BP512=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/ab8/bench64_bp512.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/ab8/bench64_def.txt 2>&1 || exit $?
