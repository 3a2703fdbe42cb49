#!/bin/bash
# deeper LDS-DMA pipelines (4 / 6 stages) for the 64-position-block forward/dgrad of small grids (NIDT_FWD_NST):
# numerics under 6 stages, then CIFAR SubAvg rounds and the per-layer ResNet bench at 10 clients
set -o pipefail
mkdir -p gpurun_out/r3ac
export PYTHONUNBUFFERED=1
NIDT_FWD_NST=6 timeout -k 10 400 python -u -m pytest tests/test_gpu_resnet2d.py tests/test_gpu_kernels.py -x -q --timeout 200 \
  --timeout-method thread -k "resnet or fwd or conv3d or graph" > gpurun_out/r3ac/pytest.txt 2>&1
rc=$?; tail -1 gpurun_out/r3ac/pytest.txt; if [ $rc -ne 0 ]; then tail -30 gpurun_out/r3ac/pytest.txt; exit $rc; fi
for arm in 6 3 4 6 3; do
  export NIDT_FWD_NST=$arm
  timeout -k 10 200 python -u tools/bench_cifar.py --algorithm subavg --rounds 2 --warmup 1 > gpurun_out/r3ac/subavg_$arm.txt 2>&1 || exit 1
  echo "subavg nst $arm: $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3ac/subavg_$arm.txt)"
done
for arm in 6 3; do
  export NIDT_FWD_NST=$arm
  timeout -k 10 200 python -u tools/kbench_resnet.py 10 > gpurun_out/r3ac/kbr_$arm.txt 2>&1 || exit 1
  echo "kbench_resnet nst $arm: $(grep 'full lockstep' gpurun_out/r3ac/kbr_$arm.txt)"
done
