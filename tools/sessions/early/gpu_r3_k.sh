#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3k
export PYTHONUNBUFFERED=1
for d in "21 25 21 1" "21 26 22 2"; do
  echo "== $d"; timeout -k 10 120 python -u tools/debug/stem_debug.py $d || exit $?
done > gpurun_out/r3k/stem_debug.txt 2>&1
rc=$?; grep -v "amdgpu.ids\|UserWarning\|Consider using\|return float" gpurun_out/r3k/stem_debug.txt; exit $rc
