#!/bin/bash
# 512-position slab blocks for the padded data gradient (NIDT_SLAB_BP=512) vs 256: numerics + kbench A/B
set -o pipefail
mkdir -p gpurun_out/r3w
export PYTHONUNBUFFERED=1 KBENCH_EVAL=0
NIDT_SLAB_BP=512 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q --timeout 120 --timeout-method thread \
  -k "slab_matches" > gpurun_out/r3w/pytest512.txt 2>&1
grep -E "passed|failed" gpurun_out/r3w/pytest512.txt | tail -2
grep -c "PASSED\|FAILED" gpurun_out/r3w/pytest512.txt
NIDT_SLAB_BP=512 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q --timeout 120 --timeout-method thread \
  -k "alexnet_train_step" > gpurun_out/r3w/pytest512b.txt 2>&1 || { tail -20 gpurun_out/r3w/pytest512b.txt; exit 1; }
tail -1 gpurun_out/r3w/pytest512b.txt
for arm in 512 256 512 256; do
  export NIDT_SLAB_BP=$arm
  timeout -k 10 300 python -u tools/kbench.py 64 10 > gpurun_out/r3w/kbench_$arm.txt 2>&1 || exit 1
  echo "arm $arm: $(grep -E 'full train step|conv2_dgrad' gpurun_out/r3w/kbench_$arm.txt | tr -s ' ' | tr '\n' ' ')"
done
