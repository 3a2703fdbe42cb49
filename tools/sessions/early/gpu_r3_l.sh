#!/bin/bash
# stem parity with native (non-MIOpen) BN reference; conv1 wgrad with single ds_read_b64 LDS reads: UNR A/B
set -o pipefail
mkdir -p gpurun_out/r3l
export PYTHONUNBUFFERED=1
timeout -k 10 100 python -u tools/debug/stem_debug.py 21 26 22 2 2>&1 | grep -v "amdgpu.ids\|UserWarning\|Consider using\|return float" > gpurun_out/r3l/stem_debug_native.txt || exit 1
head -8 gpurun_out/r3l/stem_debug_native.txt
timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_resnet3d.py -k "stem or lockstep" \
  > gpurun_out/r3l/pytest_resnet3d.txt 2>&1
rc=$?; tail -6 gpurun_out/r3l/pytest_resnet3d.txt; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread \
  -k "conv1 or alexnet" > gpurun_out/r3l/pytest_kernels.txt 2>&1 || { tail -20 gpurun_out/r3l/pytest_kernels.txt; exit 1; }
tail -2 gpurun_out/r3l/pytest_kernels.txt
for u in 1 2 4 1; do
  export NIDT_C1WG_UNROLL=$u
  timeout -k 10 300 python -u tools/kbench.py 64 10 > gpurun_out/r3l/kbench_u$u.txt 2>&1 || exit 1
  echo "== unroll $u"; grep -E "full train step|conv1_wgrad" gpurun_out/r3l/kbench_u$u.txt
done
