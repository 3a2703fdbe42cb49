#!/bin/bash
# full GPU suite with per-test durations (budget audit), then the smoke
set -o pipefail
mkdir -p gpurun_out/r4g
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread --durations=60 \
  > gpurun_out/r4g/pytest_gpu.txt 2>&1; rc=$?
tail -75 gpurun_out/r4g/pytest_gpu.txt
exit $rc
