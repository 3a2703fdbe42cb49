#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3i
export PYTHONUNBUFFERED=1
for d in "21 26 22 2" "21 26 22 1" "21 25 21 2" "121 145 121 1"; do
  echo "== $d"; timeout -k 10 120 python -u tools/debug/stem_debug.py $d || exit $?
done > gpurun_out/r3i/stem_debug.txt 2>&1
rc=$?; cat gpurun_out/r3i/stem_debug.txt | grep -v amdgpu.ids; exit $rc
