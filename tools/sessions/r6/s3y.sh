#!/bin/bash
# rerun of the ResNet graphs-vs-eager bit-identity test alone and after the kernel/resnet3d test files
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s3y; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_resnet2d.py -k graphs_match_eager > $OUT/t1.txt 2>&1; echo "alone rc=$?"; tail -1 $OUT/t1.txt
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_resnet2d.py > $OUT/t2.txt 2>&1; echo "file rc=$?"; tail -1 $OUT/t2.txt
