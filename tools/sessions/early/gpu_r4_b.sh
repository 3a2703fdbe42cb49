#!/bin/bash
# round 4, call b: 32x32 smfmac probe, smfmac conv1 wgrad vs VALU test, kbench A/B of the two conv1 wgrad kernels
set -o pipefail
mkdir -p gpurun_out/r4b
timeout -k 10 60 tools/probes/smfmac_probe gpurun_out/r4b > gpurun_out/r4b/probe.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "smfmac or conv1_fused" > gpurun_out/r4b/pytest.txt 2>&1 || { tail -40 gpurun_out/r4b/pytest.txt; exit 1; }
tail -5 gpurun_out/r4b/pytest.txt
for mode in 0 1 0 1; do
  NIDT_C1WG_SMF=$mode timeout -k 10 200 python tools/kbench.py 64 10 > gpurun_out/r4b/kbench_g64_smf$mode.txt 2>&1 || exit 1
  echo "smf=$mode"; grep -E "full train|conv1_wgrad" gpurun_out/r4b/kbench_g64_smf$mode.txt
done
for mode in 0 1; do
  NIDT_C1WG_SMF=$mode timeout -k 10 200 python tools/kbench.py 8 10 > gpurun_out/r4b/kbench_g8_smf$mode.txt 2>&1 || exit 1
  echo "g8 smf=$mode"; grep -E "full train|conv1_wgrad" gpurun_out/r4b/kbench_g8_smf$mode.txt
done
