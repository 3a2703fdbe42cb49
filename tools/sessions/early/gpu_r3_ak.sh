#!/bin/bash
# vectorized pack kernels in the ResNet engines: numerics + CIFAR SubAvg / DisPFL / Tiny rounds
set -o pipefail
mkdir -p gpurun_out/r3ak
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_resnet2d.py tests/test_gpu_resnet3d.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r3ak/pytest.txt 2>&1
rc=$?; tail -1 gpurun_out/r3ak/pytest.txt; if [ $rc -ne 0 ]; then tail -30 gpurun_out/r3ak/pytest.txt; exit $rc; fi
for a in subavg dispfl; do
  timeout -k 10 300 python -u tools/bench_cifar.py --algorithm $a --rounds 2 --warmup 1 > gpurun_out/r3ak/$a.txt 2>&1 || exit 1
  grep '^{' gpurun_out/r3ak/$a.txt | cut -c1-200
done
timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg --dataset tiny --batch 128 --rounds 2 --warmup 1 > gpurun_out/r3ak/tiny.txt 2>&1 || exit 1
grep '^{' gpurun_out/r3ak/tiny.txt | cut -c1-200
