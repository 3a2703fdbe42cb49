#!/bin/bash
# row-batched no-LDS pack for the 1x1 layers (NIDT_PACK1): ResNet engine numerics, then config 5 and CIFAR A/B
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4x; mkdir -p $OUT
NIDT_PACK1=1 timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_resnet2d.py \
  tests/test_gpu_resnet3d.py tests/test_gpu_kernels.py -k "resnet or gconv or pack or bottleneck" \
  > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for arm in 1 0; do
  NIDT_PACK1=$arm timeout -k 10 400 python3 -u tools/config5_resnet3d.py --clients 256 --train-per-client 36 \
    --test-per-client 9 --batch 4 --group 32 --rounds 3 --warmup 1 > $OUT/config5_p$arm.txt 2>&1 \
    || { tail -30 $OUT/config5_p$arm.txt; exit 1; }
  echo "config5 pack1=$arm: $(grep '^{' $OUT/config5_p$arm.txt | grep -o '"s_round_each": [^]]*]')"
done
for arm in 1 0 1b 0b; do
  v=${arm%b}
  NIDT_PACK1=$v timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg --rounds 3 --warmup 1 \
    > $OUT/subavg_p$arm.txt 2>&1 || { tail -5 $OUT/subavg_p$arm.txt; exit 1; }
  echo "subavg pack1=$arm: $(grep -o '"s_round_each": [^]]*]' $OUT/subavg_p$arm.txt)"
done
