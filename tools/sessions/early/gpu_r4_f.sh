#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r4f
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "smfmac" > gpurun_out/r4f/pytest.txt 2>&1 || { tail -30 gpurun_out/r4f/pytest.txt; exit 1; }
tail -2 gpurun_out/r4f/pytest.txt
for mode in 0 1; do
  NIDT_C1WG_SMF=$mode timeout -k 10 200 python tools/kbench.py 64 10 > gpurun_out/r4f/kbench_g64_smf$mode.txt 2>&1 || exit 1
  echo "smf=$mode"; grep -E "full train|conv1_wgrad" gpurun_out/r4f/kbench_g64_smf$mode.txt
done
