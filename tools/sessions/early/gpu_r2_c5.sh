#!/bin/bash
# config 5 (3D ResNet-50, full res): GPU tests of the client-batched engine, then 32- and 256-client rounds
set -o pipefail
mkdir -p gpurun_out/c5
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_resnet3d.py \
  > gpurun_out/c5/pytest.txt 2>&1 || { tail -40 gpurun_out/c5/pytest.txt; exit 1; }
tail -3 gpurun_out/c5/pytest.txt
timeout -k 10 400 python -u tools/config5_resnet3d.py --clients 32 --rounds 3 --engine hip > gpurun_out/c5/hip32.txt 2>&1 \
  || { tail -20 gpurun_out/c5/hip32.txt; exit 1; }
grep '^{' gpurun_out/c5/hip32.txt
