#!/bin/bash
# BASELINE config 5 on one MI355X: 3D ResNet-50 full-res, 32 clients, sparse top-k all-gather path; 3 rounds
# (round 0 includes MIOpen's kernel search), with the 3x3x3 convs on the HIP kernels and, for comparison, on MIOpen.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python tools/config5_resnet3d.py --clients 32 --rounds 3 > gpurun_out/config5.txt 2>&1 || exit $?
timeout -k 10 500 python tools/config5_resnet3d.py --clients 32 --rounds 3 --no-hip-convs > gpurun_out/config5_miopen.txt 2>&1 || exit $?
