#!/bin/bash
# 1x1x1 convs of the 3D ResNet on batched hipBLASLt GEMMs (NIDT_R3D_BLAS): engine numerics, then config 5
# (256 clients, 3 rounds) with and without, interleaved
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4t; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_resnet3d.py \
  tests/test_gpu_kernels.py -k "resnet3d or gconv or bottleneck" > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for arm in 1 0; do
  NIDT_R3D_BLAS=$arm timeout -k 10 400 python3 -u tools/config5_resnet3d.py --clients 256 --train-per-client 36 \
    --test-per-client 9 --batch 4 --group 32 --rounds 3 --warmup 1 > $OUT/config5_blas$arm.txt 2>&1 \
    || { tail -30 $OUT/config5_blas$arm.txt; exit 1; }
  echo "blas=$arm: $(grep '^{' $OUT/config5_blas$arm.txt | grep -o '"steady_s_per_round": [0-9.]*\|"s_round_each": [^]]*]\|"peak_gib_each_round": [^]]*]\|"phase_s_each_round": [^]]*]' | tr '\n' ' ')"
done
