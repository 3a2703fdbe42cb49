#!/bin/bash
# kd-slab union forward (k_conv_fwd_slab): kernel tests, then kbench A/B (NIDT_FWD_SLAB=1: conv2 dgrad, =2: + conv2 fwd, =0 off)
set -o pipefail
mkdir -p gpurun_out/r3v
export PYTHONUNBUFFERED=1 KBENCH_EVAL=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "slab or fwd_stats or alexnet or graph" > gpurun_out/r3v/pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r3v/pytest.txt; if [ $rc -ne 0 ]; then exit $rc; fi
for arm in 1 0 2 1 0 2; do
  export NIDT_FWD_SLAB=$arm
  timeout -k 10 300 python -u tools/kbench.py 64 10 > gpurun_out/r3v/kbench_$arm.txt 2>&1 || exit 1
  echo "arm $arm: $(grep -E 'full train step|conv2_fwd|conv2_dgrad' gpurun_out/r3v/kbench_$arm.txt | tr '\n' ' ')"
done
