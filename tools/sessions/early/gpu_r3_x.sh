#!/bin/bash
# kd-slab union wgrad (k_conv_wgrad_slab): numerics, then kbench A/B (NIDT_WG_SLAB=1 where tri was chosen, 0 = tri)
set -o pipefail
mkdir -p gpurun_out/r3x
export PYTHONUNBUFFERED=1 KBENCH_EVAL=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "wgrad_slab or alexnet_train_step or graph" > gpurun_out/r3x/pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r3x/pytest.txt; if [ $rc -ne 0 ]; then exit $rc; fi
for arm in 1 0 1 0; do
  export NIDT_WG_SLAB=$arm
  timeout -k 10 300 python -u tools/kbench.py 64 10 > gpurun_out/r3x/kbench_$arm.txt 2>&1 || exit 1
  echo "arm $arm: $(grep -E 'full train step|_wgrad' gpurun_out/r3x/kbench_$arm.txt | tr -s ' ' | tr '\n' '|')"
done
