#!/bin/bash
# split-K general forward: numerics (2-D + 3-D ResNet engines), per-layer A/B (NIDT_FWDG_KSPLIT=1 = off), CIFAR bench A/B
set -o pipefail
mkdir -p gpurun_out/sk
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_resnet2d.py tests/test_gpu_resnet3d.py > gpurun_out/sk/pytest.txt 2>&1 || { tail -30 gpurun_out/sk/pytest.txt; exit 1; }
tail -1 gpurun_out/sk/pytest.txt
for G in 100 10; do
  timeout -k 10 200 python -u tools/kbench_resnet.py $G 10 > gpurun_out/sk/kb_on_$G.txt 2>&1 || exit 1
  NIDT_FWDG_KSPLIT=1 timeout -k 10 200 python -u tools/kbench_resnet.py $G 10 > gpurun_out/sk/kb_off_$G.txt 2>&1 || exit 1
done
grep -E "conv|step" gpurun_out/sk/kb_*.txt
timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg > gpurun_out/sk/cifar_on.txt 2>&1 || exit 1
NIDT_FWDG_KSPLIT=1 timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg > gpurun_out/sk/cifar_off.txt 2>&1 || exit 1
grep '^{' gpurun_out/sk/cifar_*.txt | cut -c1-300
