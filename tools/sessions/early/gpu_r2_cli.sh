#!/bin/bash
# CLI routing of the ResNet families onto the client-batched HIP engines
set -o pipefail
mkdir -p gpurun_out/cli
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cli.py -k "resnet" > gpurun_out/cli/pytest.txt 2>&1 || { tail -40 gpurun_out/cli/pytest.txt; exit 1; }
tail -12 gpurun_out/cli/pytest.txt
