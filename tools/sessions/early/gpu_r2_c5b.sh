#!/bin/bash
# config 5 at 256 clients: client-batched HIP engine vs the per-client all-MIOpen TorchEngine path
set -o pipefail
mkdir -p gpurun_out/c5
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u tools/config5_resnet3d.py --clients 256 --rounds 2 --engine hip > gpurun_out/c5/hip256.txt 2>&1 \
  || { tail -20 gpurun_out/c5/hip256.txt; exit 1; }
grep '^{' gpurun_out/c5/hip256.txt
timeout -k 10 600 python -u tools/config5_resnet3d.py --clients 256 --rounds 2 --engine torch --no-hip-convs > gpurun_out/c5/miopen256.txt 2>&1 \
  || { tail -20 gpurun_out/c5/miopen256.txt; exit 1; }
grep '^{' gpurun_out/c5/miopen256.txt
