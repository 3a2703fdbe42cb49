#!/bin/bash
# conv1 fused forward with the dd loop unrolled (NIDT_C1_DDU=3) vs rolled: numerics + kbench A/B
set -o pipefail
mkdir -p gpurun_out/r3aa
export PYTHONUNBUFFERED=1 KBENCH_EVAL=0
NIDT_C1_DDU=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "conv1 or alexnet" > gpurun_out/r3aa/pytest.txt 2>&1
rc=$?; tail -1 gpurun_out/r3aa/pytest.txt; if [ $rc -ne 0 ]; then exit $rc; fi
for arm in 3 1 3 1; do
  export NIDT_C1_DDU=$arm
  timeout -k 10 300 python -u tools/kbench.py 64 10 > gpurun_out/r3aa/kbench_$arm.txt 2>&1 || exit 1
  echo "arm $arm: $(grep -E 'full train step|conv1_fwd' gpurun_out/r3aa/kbench_$arm.txt | tr -s ' ' | tr '\n' '|')"
done
