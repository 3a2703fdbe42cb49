#!/bin/bash
# batched-depth slab: correctness test, kernel bench, then SubAvg profile
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5l2; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_resnet2d.py -k "slab_batched_depth" > $OUT/pytest.txt 2>&1 || { grep -E "Error|assert|FAILED|passed|failed" $OUT/pytest.txt | tail -20; exit 1; }
tail -1 $OUT/pytest.txt
bash tools/sessions/r5/a2.sh && bash tools/sessions/r5/k2.sh
