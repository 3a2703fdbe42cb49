#!/bin/bash
# ResNet-18-GN (CIFAR) HIP path: GPU tests, graph-replay poison check, then the reference evidence configs
# (SubAvg / DisPFL, 100 clients).
set -o pipefail
mkdir -p gpurun_out/resnet
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_resnet2d.py \
  > gpurun_out/resnet/pytest.txt 2>&1 || { tail -40 gpurun_out/resnet/pytest.txt; exit 1; }
tail -3 gpurun_out/resnet/pytest.txt
cat gpurun_out/resnet/graph_poison.txt | grep -v amdgpu.ids
timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg --rounds 2 --warmup 1 \
  > gpurun_out/resnet/bench_subavg.txt 2>&1 || { tail -30 gpurun_out/resnet/bench_subavg.txt; exit 1; }
tail -4 gpurun_out/resnet/bench_subavg.txt
timeout -k 10 400 python -u tools/bench_cifar.py --algorithm dispfl --rounds 1 --warmup 1 \
  > gpurun_out/resnet/bench_dispfl.txt 2>&1 || { tail -30 gpurun_out/resnet/bench_dispfl.txt; exit 1; }
tail -4 gpurun_out/resnet/bench_dispfl.txt
