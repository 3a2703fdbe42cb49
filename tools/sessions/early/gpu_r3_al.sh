#!/bin/bash
# pack-kernel vectorization A/B on the ResNet engines: current build vs the previous one (tools/ab_so), interleaved
set -o pipefail
mkdir -p gpurun_out/r3al /tmp/oldext
cp tools/ab_so/_nidt_hip_old.so /tmp/oldext/_nidt_hip.cpython-310-x86_64-linux-gnu.so
export PYTHONUNBUFFERED=1
for arm in new old new old; do
  if [ $arm = old ]; then export NIDT_EXT_DIR=/tmp/oldext; else unset NIDT_EXT_DIR; fi
  timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg --dataset tiny --batch 128 --rounds 2 --warmup 1 > gpurun_out/r3al/tiny_$arm.txt 2>&1 || exit 1
  echo "tiny $arm: $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3al/tiny_$arm.txt)"
  timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg --rounds 2 --warmup 1 > gpurun_out/r3al/subavg_$arm.txt 2>&1 || exit 1
  echo "subavg $arm: $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3al/subavg_$arm.txt)"
done
