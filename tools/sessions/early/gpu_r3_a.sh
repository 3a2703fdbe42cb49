#!/bin/bash
# round 3, first box: the new ResNet-2D / runner paths, then the headline bench
set -o pipefail
mkdir -p gpurun_out/r3a
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_resnet2d.py tests/test_gpu_runner.py -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/r3a/pytest_new.txt 2>&1
rc=$?; tail -3 gpurun_out/r3a/pytest_new.txt; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r3a/bench.txt 2>&1 || exit 1
grep '^{' gpurun_out/r3a/bench.txt | cut -c1-400
