#!/bin/bash
# bisect the first-in-process DisPFL graphs-vs-eager mismatch over the round-6 switches
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s3z; mkdir -p $OUT
i=0
for e in X=0 NIDT_FORK_GROUP=0 NIDT_STEM_FOLD=0 "NIDT_GN_RMASK=0 NIDT_OMASK2D=0" NIDT_GN_HOLD=4 NIDT_WGRAD_STREAM=0 X=1; do
  i=$((i+1))
  env $e timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_resnet2d.py -k graphs_match_eager > $OUT/t_$i.txt 2>&1; rc=$?
  echo "== $e rc=$rc $(tail -1 $OUT/t_$i.txt)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
done
