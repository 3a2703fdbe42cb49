#!/bin/bash
# whole-sample union conv (k_conv_fwd_vol) for the AlexNet conv3-5 forward / data gradient: numerics, then kbench at
# 64 and 8 clients, arms interleaved (NIDT_FWD_VOL=1 / 0; WM=2 variant)
set -o pipefail
mkdir -p gpurun_out/r3aw
export PYTHONUNBUFFERED=1 KBENCH_EVAL=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread \
  -k "vol or alexnet or stats or step" > gpurun_out/r3aw/pytest.txt 2>&1
rc=$?; tail -1 gpurun_out/r3aw/pytest.txt; if [ $rc -ne 0 ]; then grep -E "Error|assert|FAIL" gpurun_out/r3aw/pytest.txt | head -30; exit $rc; fi
for arm in 1 0 1 0 w2; do
  if [ $arm = w2 ]; then export NIDT_FWD_VOL=1 NIDT_FWD_VOL_WM=2; else export NIDT_FWD_VOL=$arm; unset NIDT_FWD_VOL_WM; fi
  timeout -k 10 300 python -u tools/kbench.py 64 10 > gpurun_out/r3aw/kb64_$arm.txt 2>&1 || { tail -20 gpurun_out/r3aw/kb64_$arm.txt; exit 1; }
  echo "vol=$arm G64: $(grep -E 'full train step|conv[345]_(fwd|dgrad)' gpurun_out/r3aw/kb64_$arm.txt | tr -s ' ' | cut -c1-60 | tr '\n' '|')"
done
for arm in 1 0; do
  export NIDT_FWD_VOL=$arm; unset NIDT_FWD_VOL_WM
  timeout -k 10 300 python -u tools/kbench.py 8 10 > gpurun_out/r3aw/kb8_$arm.txt 2>&1 || { tail -20 gpurun_out/r3aw/kb8_$arm.txt; exit 1; }
  echo "vol=$arm G8: $(grep -E 'full train step|conv[345]_(fwd|dgrad)' gpurun_out/r3aw/kb8_$arm.txt | tr -s ' ' | cut -c1-60 | tr '\n' '|')"
done
