#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5q; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_resnet3d.py -k "stem" > $OUT/t.txt 2>&1 || { grep -E "FAIL|Error|assert|error" $OUT/t.txt | tail -40; exit 1; }
tail -1 $OUT/t.txt
timeout -k 10 200 python -u tools/bench_stem.py > $OUT/stem.txt 2>&1 || { tail -20 $OUT/stem.txt; exit 1; }
grep stem_pool $OUT/stem.txt
