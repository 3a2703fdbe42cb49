#!/bin/bash
# GroupNorm channel reduction with wave shuffles: GN / ResNet tests, then interleaved A/B against the previous build
# (NIDT_EXT_DIR = tools/ab_so) on CIFAR SubAvg / DisPFL and Tiny SubAvg at tiny.sh's batch 128
set -o pipefail
mkdir -p gpurun_out/r3ba /tmp/oldext
cp tools/ab_so/_nidt_hip_old.so /tmp/oldext/_nidt_hip.cpython-310-x86_64-linux-gnu.so
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_resnet2d.py tests/test_gpu_resnet3d.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/r3ba/pytest.txt 2>&1
rc=$?; tail -1 gpurun_out/r3ba/pytest.txt; if [ $rc -ne 0 ]; then grep -E "Error|assert|FAIL" gpurun_out/r3ba/pytest.txt | head -30; exit $rc; fi
for arm in new old new old; do
  if [ $arm = old ]; then export NIDT_EXT_DIR=/tmp/oldext; else unset NIDT_EXT_DIR; fi
  timeout -k 10 200 python -u tools/bench_cifar.py --algorithm subavg --rounds 2 --warmup 1 > gpurun_out/r3ba/subavg_$arm.txt 2>&1 || exit 1
  echo "$arm: subavg $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3ba/subavg_$arm.txt)"
done
for arm in new old; do
  if [ $arm = old ]; then export NIDT_EXT_DIR=/tmp/oldext; else unset NIDT_EXT_DIR; fi
  timeout -k 10 300 python -u tools/bench_cifar.py --algorithm dispfl --rounds 1 --warmup 1 > gpurun_out/r3ba/dispfl_$arm.txt 2>&1 || exit 1
  echo "$arm: dispfl $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3ba/dispfl_$arm.txt)"
  timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg --dataset tiny --batch 128 --rounds 1 --warmup 1 > gpurun_out/r3ba/tiny_$arm.txt 2>&1 || exit 1
  echo "$arm: tiny subavg b128 $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3ba/tiny_$arm.txt)"
done
