#!/bin/bash
# k-split wave groups in the small-grid forward/dgrad blocks (NIDT_FWD_KW = 2 / 4): numerics, CIFAR SubAvg, AlexNet G=8
set -o pipefail
mkdir -p gpurun_out/r3aq
export PYTHONUNBUFFERED=1
for kw in 2 4; do
  NIDT_FWD_KW=$kw timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_resnet2d.py -x -q --timeout 200 \
    --timeout-method thread -k "conv or resnet or graph or alexnet" > gpurun_out/r3aq/pytest_$kw.txt 2>&1
  rc=$?; echo "kw $kw: $(tail -1 gpurun_out/r3aq/pytest_$kw.txt)"; if [ $rc -ne 0 ]; then tail -30 gpurun_out/r3aq/pytest_$kw.txt; exit $rc; fi
done
for arm in 2 1 4 2 1 4; do
  export NIDT_FWD_KW=$arm
  timeout -k 10 200 python -u tools/bench_cifar.py --algorithm subavg --rounds 2 --warmup 1 > gpurun_out/r3aq/subavg_$arm.txt 2>&1 || exit 1
  echo "subavg kw $arm: $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3aq/subavg_$arm.txt)"
done
for arm in 2 1 4 2 1 4; do
  export NIDT_FWD_KW=$arm
  timeout -k 10 200 python -u bench.py --clients 8 --steps 15 --warmup 3 > gpurun_out/r3aq/b8_$arm.txt 2>&1 || exit 1
  echo "alexnet 8 clients kw $arm: $(grep -o '"value": [0-9.]*' gpurun_out/r3aq/b8_$arm.txt)"
done
