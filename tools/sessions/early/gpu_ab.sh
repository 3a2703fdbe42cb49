#!/bin/bash
# A/B of a kernel-selection change: numerics tests, then kbench + 1-GPU bench with the new rule and with
# NIDT_WG_NSPLIT_LEGACY=1, at 64 and 8 clients.
set -o pipefail
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "${PYTEST_K:-conv3d or alexnet or head}" > gpurun_out/ab/pytest.txt 2>&1 || exit $?
for G in 64 8; do
  timeout -k 10 200 python tools/kbench.py $G 10 > gpurun_out/ab/kbench${G}_new.txt 2>&1 || exit $?
  NIDT_WG_NSPLIT_LEGACY=1 timeout -k 10 200 python tools/kbench.py $G 10 > gpurun_out/ab/kbench${G}_old.txt 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/ab/bench64_new.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --clients 8 --steps 10 --warmup 3 > gpurun_out/ab/bench8_new.txt 2>&1 || exit $?
NIDT_WG_NSPLIT_LEGACY=1 timeout -k 10 300 python bench.py --clients 8 --steps 10 --warmup 3 > gpurun_out/ab/bench8_old.txt 2>&1 || exit $?
