#!/bin/bash
# conv1 forward with the 128-slot K layout: numerics (GPU kernel tests) + kbench A/B against the 224-slot layout
set -o pipefail
mkdir -p gpurun_out/r3b
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3b/pytest_kernels.txt 2>&1
rc=$?; tail -3 gpurun_out/r3b/pytest_kernels.txt; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
for arm in 128 224 128; do
  if [ $arm = 224 ]; then export NIDT_C1_K224=1; else unset NIDT_C1_K224; fi
  timeout -k 10 300 python -u tools/kbench.py 64 10 > gpurun_out/r3b/kbench_$arm.txt 2>&1 || exit 1
  echo "== K slots $arm"; grep -E "full train step|conv1|eval" gpurun_out/r3b/kbench_$arm.txt
done
unset NIDT_C1_K224
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r3b/bench.txt 2>&1 || exit 1
grep '^{' gpurun_out/r3b/bench.txt | cut -c1-300
