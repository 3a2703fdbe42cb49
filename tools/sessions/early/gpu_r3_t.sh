#!/bin/bash
# ResNet engines with the weight-gradient branch stream: GPU tests, then CIFAR SubAvg / DisPFL / Tiny A/B (NIDT_WGRAD_STREAM)
set -o pipefail
mkdir -p gpurun_out/r3t
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_resnet2d.py tests/test_gpu_resnet3d.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/r3t/pytest.txt 2>&1
rc=$?; tail -2 gpurun_out/r3t/pytest.txt; if [ $rc -ne 0 ]; then exit $rc; fi
for arm in 1 0 1 0; do
  export NIDT_WGRAD_STREAM=$arm
  timeout -k 10 200 python -u tools/bench_cifar.py --algorithm subavg --rounds 2 --warmup 1 > gpurun_out/r3t/subavg_$arm.txt 2>&1 || exit 1
  echo "subavg arm $arm: $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3t/subavg_$arm.txt)"
done
for arm in 1 0; do
  export NIDT_WGRAD_STREAM=$arm
  timeout -k 10 200 python -u tools/bench_cifar.py --algorithm dispfl --rounds 2 --warmup 1 > gpurun_out/r3t/dispfl_$arm.txt 2>&1 || exit 1
  echo "dispfl arm $arm: $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3t/dispfl_$arm.txt)"
  timeout -k 10 200 python -u tools/bench_cifar.py --algorithm subavg --dataset tiny --batch 128 --rounds 2 --warmup 1 > gpurun_out/r3t/tiny_$arm.txt 2>&1 || exit 1
  echo "tiny arm $arm: $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3t/tiny_$arm.txt)"
done
