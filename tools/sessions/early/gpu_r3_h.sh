#!/bin/bash
# conv1 sparse wgrad with cell-paired bf16 dot products (k_conv1_wgrad_dot): numerics (GPU kernel tests, both
# kernels) + kbench A/B against the v_pk_fma_f32 kernel, then the bench
set -o pipefail
mkdir -p gpurun_out/r3h
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 200 --timeout-method thread \
  -k "conv1 or alexnet" > gpurun_out/r3h/pytest_dot.txt 2>&1
rc=$?; tail -3 gpurun_out/r3h/pytest_dot.txt; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
for arm in dot pk dot; do
  if [ $arm = pk ]; then export NIDT_C1WG_DOT=0; else unset NIDT_C1WG_DOT; fi
  timeout -k 10 300 python -u tools/kbench.py 64 10 > gpurun_out/r3h/kbench_$arm.txt 2>&1 || exit 1
  echo "== wgrad $arm"; grep -E "full train step|conv1" gpurun_out/r3h/kbench_$arm.txt
done
unset NIDT_C1WG_DOT
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r3h/bench.txt 2>&1 || exit 1
grep '^{' gpurun_out/r3h/bench.txt | cut -c1-300
