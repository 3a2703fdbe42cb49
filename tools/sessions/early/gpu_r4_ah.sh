#!/bin/bash
# extended GPU shape sweeps (NIDT_EXTENDED_GPU_TESTS=1) of the kernel and ResNet suites on the schedule-changed conv
# kernels (default switches)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4ah; mkdir -p $OUT
NIDT_EXTENDED_GPU_TESTS=1 timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_resnet2d.py tests/test_gpu_resnet3d.py -m gpu > $OUT/pytest_ext.txt 2>&1 \
  || { grep -E "FAILED|Error|passed|failed" $OUT/pytest_ext.txt | tail -20; exit 1; }
grep -E "passed|failed" $OUT/pytest_ext.txt | tail -1
