#!/bin/bash
# round-3 Tiny / CIFAR round-time diagnosis (the session-3 switches one at a time, interleaved)
set -o pipefail
mkdir -p gpurun_out/r4k
bash tools/sessions/early/gpu_r3_bc.sh 2>&1 | tee gpurun_out/r4k/r3bc.txt
cp -r gpurun_out/r3bc gpurun_out/r4k/ 2>/dev/null
true
