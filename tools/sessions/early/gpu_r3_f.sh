#!/bin/bash
# HIP stem (stem.hip) parity + the 3D ResNet tests, then the chaos-control cosines of the HIP-vs-fp32 runner test
set -o pipefail
mkdir -p gpurun_out/r3f
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_resnet3d.py -k "stem or lockstep" \
  > gpurun_out/r3f/pytest_resnet3d.txt 2>&1
rc=$?; tail -15 gpurun_out/r3f/pytest_resnet3d.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u tools/chaos_cosine.py fedavg salientgrads local ditto > gpurun_out/r3f/chaos.txt 2>&1
rc=$?; grep '^{' gpurun_out/r3f/chaos.txt; exit $rc
