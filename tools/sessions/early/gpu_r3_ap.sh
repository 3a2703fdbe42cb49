#!/bin/bash
# conv1 forward at 3 blocks per CU (lean register variant, NIDT_C1_OCC=3) vs 2: numerics + kbench A/B (train + eval)
set -o pipefail
mkdir -p gpurun_out/r3ap
export PYTHONUNBUFFERED=1
NIDT_C1_OCC=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "conv1 or alexnet" > gpurun_out/r3ap/pytest.txt 2>&1
rc=$?; tail -1 gpurun_out/r3ap/pytest.txt; if [ $rc -ne 0 ]; then tail -30 gpurun_out/r3ap/pytest.txt; exit $rc; fi
for arm in 3 2 3 2; do
  export NIDT_C1_OCC=$arm
  timeout -k 10 300 python -u tools/kbench.py 64 10 > gpurun_out/r3ap/kbench_$arm.txt 2>&1 || exit 1
  echo "arm $arm: $(grep -E 'full train step|conv1_fwd|eval forward' gpurun_out/r3ap/kbench_$arm.txt | tr -s ' ' | cut -c1-150 | tr '\n' '|')"
done
