#!/bin/bash
# fused ResNet classifier head (cls_head_train): numerics vs the torch head, interleaved CIFAR / Tiny A/B (NIDT_CLS_HEAD)
set -o pipefail
mkdir -p gpurun_out/r3av
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_resnet2d.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r3av/pytest.txt 2>&1
rc=$?; tail -1 gpurun_out/r3av/pytest.txt; if [ $rc -ne 0 ]; then tail -40 gpurun_out/r3av/pytest.txt; exit $rc; fi
for arm in 1 0 1 0; do
  export NIDT_CLS_HEAD=$arm
  timeout -k 10 200 python -u tools/bench_cifar.py --algorithm subavg --rounds 2 --warmup 1 > gpurun_out/r3av/subavg_$arm.txt 2>&1 || exit 1
  echo "head=$arm: subavg $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3av/subavg_$arm.txt)"
done
for arm in 1 0; do
  export NIDT_CLS_HEAD=$arm
  timeout -k 10 300 python -u tools/bench_cifar.py --algorithm dispfl --rounds 1 --warmup 1 > gpurun_out/r3av/dispfl_$arm.txt 2>&1 || exit 1
  echo "head=$arm: dispfl $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3av/dispfl_$arm.txt)"
done
for arm in 1 0; do
  export NIDT_CLS_HEAD=$arm
  timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg --dataset tiny --rounds 1 --warmup 1 > gpurun_out/r3av/tiny_$arm.txt 2>&1 || exit 1
  echo "head=$arm: tiny subavg $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3av/tiny_$arm.txt)"
done
