#!/bin/bash
# smfmac conv1 wgrad v4 (warp-specialised, double-buffered): correctness vs the VALU gather, then kbench A/B
set -o pipefail
mkdir -p gpurun_out/r4i
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "smfmac" > gpurun_out/r4i/pytest.txt 2>&1 || { tail -30 gpurun_out/r4i/pytest.txt; exit 1; }
tail -2 gpurun_out/r4i/pytest.txt
for mode in 0 1 0 1; do
  NIDT_C1WG_SMF=$mode timeout -k 10 200 python tools/kbench.py 64 10 > gpurun_out/r4i/kbench_g64_smf$mode.txt 2>&1 || exit 1
  echo "smf=$mode: $(grep -E 'full train' gpurun_out/r4i/kbench_g64_smf$mode.txt) $(grep -E '^conv1_wgrad' gpurun_out/r4i/kbench_g64_smf$mode.txt)"
done
for mode in 0 1; do
  NIDT_C1WG_SMF=$mode timeout -k 10 200 python tools/kbench.py 8 10 > gpurun_out/r4i/kbench_g8_smf$mode.txt 2>&1 || exit 1
  echo "g8 smf=$mode: $(grep -E 'full train' gpurun_out/r4i/kbench_g8_smf$mode.txt) $(grep -E '^conv1_wgrad' gpurun_out/r4i/kbench_g8_smf$mode.txt)"
done
