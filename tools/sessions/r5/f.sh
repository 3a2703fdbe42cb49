#!/bin/bash
# full GPU suite + headline bench (64 clients) + 8-client bench on the new conv1 weight-gradient default
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5k; mkdir -p $OUT
timeout -k 10 120 python -u tools/sessions/r5/fp.py > $OUT/fp.txt 2>&1 && cat $OUT/fp.txt | grep FINGER && timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu --deselect tests/test_gpu_convergence.py::test_hip_bf16_tracks_fp32_over_twenty_rounds > $OUT/pytest_gpu.txt 2>&1 \
  || { grep -E "FAILED|Error|passed|failed" $OUT/pytest_gpu.txt | tail -20; exit 1; }
tail -2 $OUT/pytest_gpu.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench64.txt 2>&1 || { tail -20 $OUT/bench64.txt; exit 1; }
tail -1 $OUT/bench64.txt
timeout -k 10 300 python -u bench.py --clients 8 --steps 30 --warmup 5 > $OUT/bench8.txt 2>&1 || exit 1
tail -1 $OUT/bench8.txt
