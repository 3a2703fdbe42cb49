#!/bin/bash
# A/B: forward/dgrad LDS-DMA pipeline depth on small grids (default: 3 stages when < 2 blocks per CU) vs
# NIDT_FWD_NST=2 everywhere; numerics tests first.
set -o pipefail
mkdir -p gpurun_out/ab2
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "${PYTEST_K:-conv3d or alexnet or head or hip_conv}" > gpurun_out/ab2/pytest.txt 2>&1 || exit $?
for G in 8 64; do
  timeout -k 10 200 python tools/kbench.py $G 10 > gpurun_out/ab2/kbench${G}_new.txt 2>&1 || exit $?
  NIDT_FWD_NST=2 timeout -k 10 200 python tools/kbench.py $G 10 > gpurun_out/ab2/kbench${G}_old.txt 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --clients 8 --steps 10 --warmup 3 > gpurun_out/ab2/bench8_new.txt 2>&1 || exit $?
