#!/bin/bash
# per-layer ResNet-18-GN step costs at the CIFAR tail's client counts (1, 2, 10 clients)
set -o pipefail
mkdir -p gpurun_out/r3af
export PYTHONUNBUFFERED=1
for G in 1 2 10; do
  timeout -k 10 200 python -u tools/kbench_resnet.py $G > gpurun_out/r3af/kbr_$G.txt 2>&1 || exit 1
  cat gpurun_out/r3af/kbr_$G.txt | grep -v amdgpu.ids
done
