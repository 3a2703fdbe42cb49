#!/bin/bash
# bisect: graph-vs-eager equality of the ResNet runners under the GN register kernels / direct wgrad epilogue
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5z; mkdir -p $OUT
T="tests/test_gpu_resnet2d.py::test_resnet18gn_hip_runners_graphs_match_eager"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_resnet2d.py -k groupnorm > $OUT/gn.txt 2>&1; echo "gn tests rc=$?"; tail -1 $OUT/gn.txt
for cfg in "NIDT_WG_DIRECT=1 NIDT_GN_HOLD=4" "NIDT_WG_DIRECT=0 NIDT_GN_HOLD=4" "NIDT_WG_DIRECT=1 NIDT_GN_HOLD=0" "NIDT_WG_DIRECT=0 NIDT_GN_HOLD=0"; do
  env $cfg timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread $T > $OUT/t.txt 2>&1; rc=$?
  echo "== $cfg rc=$rc"; tail -1 $OUT/t.txt
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
done
