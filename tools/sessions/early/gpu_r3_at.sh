#!/bin/bash
# 2-D slab convs (conv2d_fwd_slab) with the measured pick rule: engine tests, interleaved CIFAR SubAvg / DisPFL / Tiny
# A/B against the per-tap kernels (NIDT_2D_SLAB=0)
set -o pipefail
mkdir -p gpurun_out/r3at2
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_resnet2d.py tests/test_gpu_kernels.py -k "resnet or conv2d_fwd_slab or gn" -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r3at2/pytest.txt 2>&1
rc=$?; tail -1 gpurun_out/r3at2/pytest.txt; if [ $rc -ne 0 ]; then tail -30 gpurun_out/r3at2/pytest.txt; exit $rc; fi
for arm in 1 0 1 0; do
  export NIDT_2D_SLAB=$arm
  timeout -k 10 200 python -u tools/bench_cifar.py --algorithm subavg --rounds 2 --warmup 1 > gpurun_out/r3at2/subavg_$arm.txt 2>&1 || exit 1
  echo "slab=$arm: subavg $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3at2/subavg_$arm.txt)"
done
for arm in 1 0 1 0; do
  export NIDT_2D_SLAB=$arm
  timeout -k 10 300 python -u tools/bench_cifar.py --algorithm dispfl --rounds 1 --warmup 1 > gpurun_out/r3at2/dispfl_$arm.txt 2>&1 || exit 1
  echo "slab=$arm: dispfl $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3at2/dispfl_$arm.txt)"
done
for arm in 1 0; do
  export NIDT_2D_SLAB=$arm
  timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg --dataset tiny --rounds 1 --warmup 1 > gpurun_out/r3at2/tiny_$arm.txt 2>&1 || exit 1
  echo "slab=$arm: tiny subavg $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3at2/tiny_$arm.txt)"
done
