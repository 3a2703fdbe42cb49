#!/bin/bash
# kd-slab convs in the 3D ResNet-50 engine (layer-1/2 3x3x3 stride-1 fwd + dgrad): numerics + config-5 A/B
set -o pipefail
mkdir -p gpurun_out/r3an
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_resnet3d.py -x -q --timeout 300 \
  --timeout-method thread -k "slab or resnet3d or bottleneck or stem" > gpurun_out/r3an/pytest.txt 2>&1
rc=$?; tail -1 gpurun_out/r3an/pytest.txt; if [ $rc -ne 0 ]; then tail -30 gpurun_out/r3an/pytest.txt; exit $rc; fi
for arm in 2 0 2 0; do
  export NIDT_FWD_SLAB=$arm
  timeout -k 10 500 python3 -u tools/config5_resnet3d.py --clients 64 --train-per-client 36 --test-per-client 9 \
    --batch 4 --group 32 --rounds 2 > gpurun_out/r3an/c5_$arm.txt 2>&1 || { tail -20 gpurun_out/r3an/c5_$arm.txt; exit 1; }
  echo "config5 (64 clients) slab=$arm: $(grep '^{' gpurun_out/r3an/c5_$arm.txt | cut -c1-260)"
done
