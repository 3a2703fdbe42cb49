#!/bin/bash
# weight-gradient branch (NIDT_WGRAD_STREAM) A/B: train-step time (kbench) and bench.py rounds/s, interleaved arms
set -o pipefail
mkdir -p gpurun_out/r3s
export PYTHONUNBUFFERED=1 KBENCH_EVAL=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "alexnet or step or graph" > gpurun_out/r3s/pytest.txt 2>&1
rc=$?; tail -2 gpurun_out/r3s/pytest.txt; if [ $rc -gt 1 ]; then exit $rc; fi
for arm in 1 0 e 1 0 e; do
  if [ $arm = e ]; then export NIDT_WGRAD_STREAM=1 NIDT_WG2_EARLY=1; else export NIDT_WGRAD_STREAM=$arm NIDT_WG2_EARLY=0; fi
  timeout -k 10 300 python -u tools/kbench.py 64 6 > gpurun_out/r3s/kbench_$arm.txt 2>&1 || exit 1
  echo "arm $arm: $(grep 'full train step' gpurun_out/r3s/kbench_$arm.txt)"
done
for arm in 1 0 1 0; do
  export NIDT_WGRAD_STREAM=$arm NIDT_WG2_EARLY=0
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 > gpurun_out/r3s/bench_$arm.txt 2>&1 || exit 1
  echo "bench arm $arm: $(grep '^{' gpurun_out/r3s/bench_$arm.txt | cut -c1-120)"
done
