#!/bin/bash
# slab data gradient with a 3-slot weight-tile ring (NIDT_SLAB_NA=3) vs 2: numerics + kbench A/B
set -o pipefail
mkdir -p gpurun_out/r3ae
export PYTHONUNBUFFERED=1 KBENCH_EVAL=0
NIDT_SLAB_NA=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "slab or fwd_stats or alexnet" > gpurun_out/r3ae/pytest.txt 2>&1
rc=$?; tail -1 gpurun_out/r3ae/pytest.txt; if [ $rc -ne 0 ]; then exit $rc; fi
for arm in 3 2 3 2; do
  export NIDT_SLAB_NA=$arm
  timeout -k 10 300 python -u tools/kbench.py 64 10 > gpurun_out/r3ae/kbench_$arm.txt 2>&1 || exit 1
  echo "arm $arm: $(grep -E 'full train step|conv2_fwd|conv2_dgrad' gpurun_out/r3ae/kbench_$arm.txt | tr -s ' ' | tr '\n' '|')"
done
