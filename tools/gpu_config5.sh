#!/bin/bash
# BASELINE config 5 smoke on one MI355X: 3D ResNet-50 full-res, 32 clients, sparse top-k all-gather path.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python tools/config5_resnet3d.py --clients 32 --rounds 1 > gpurun_out/config5.txt 2>&1 || exit $?
