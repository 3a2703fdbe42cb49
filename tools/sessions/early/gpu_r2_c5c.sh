#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/c5
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u tools/config5_resnet3d.py --clients 256 --rounds 3 --engine hip > gpurun_out/c5/hip256_v2.txt 2>&1 \
  || { tail -20 gpurun_out/c5/hip256_v2.txt; exit 1; }
grep '^{' gpurun_out/c5/hip256_v2.txt
