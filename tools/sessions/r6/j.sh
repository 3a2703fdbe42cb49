#!/bin/bash
# eval-mode gradient test: determinism / stream-race check per slot layout
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6j; mkdir -p $OUT
T=tests/test_gpu_personalized.py::test_eval_mode_gradient_matches_autograd
for cfg in "NIDT_C1_TAPORD=2" "NIDT_C1_TAPORD=2" "NIDT_C1_TAPORD=0" "NIDT_C1_TAPORD=0" "NIDT_C1_TAPORD=2 HIP_LAUNCH_BLOCKING=1" "NIDT_C1_TAPORD=2 NIDT_AX_WGRAD_STREAM=0" "NIDT_C1_TAPORD=0 HIP_LAUNCH_BLOCKING=1"; do
  env $cfg timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread $T > $OUT/t.txt 2>&1; rc=$?
  echo "== $cfg rc=$rc"; tail -1 $OUT/t.txt; grep -o "AssertionError: {.\{0,160\}" $OUT/t.txt | head -1
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
done
