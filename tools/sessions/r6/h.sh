#!/bin/bash
# (1) debug conv1 p1 in the eval-mode step per slot layout; (2) k_conv_wgrad_dma asm-DMA numerics + CIFAR SubAvg
# and config-5 A/B
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6h; mkdir -p $OUT
for T in 2 0; do
  echo "== TAPORD=$T"; NIDT_C1_TAPORD=$T timeout -k 10 200 python -u tools/debug/c1_evalmode.py > $OUT/dbg_$T.txt 2>&1 || { tail -20 $OUT/dbg_$T.txt; exit 1; }
  grep -v amdgpu.ids $OUT/dbg_$T.txt
done
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_resnet2d.py tests/test_gpu_resnet3d.py -k "wgrad or resnet" > $OUT/t.txt 2>&1 || { tail -30 $OUT/t.txt; exit 1; }
tail -1 $OUT/t.txt
for A in 1 0; do
  NIDT_WGD_ADMA=$A timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg --rounds 2 --warmup 1 > $OUT/subavg_$A.txt 2>&1 || { tail -20 $OUT/subavg_$A.txt; exit 1; }
  echo "== WGD_ADMA=$A"; tail -1 $OUT/subavg_$A.txt | cut -c1-200
done
for A in 1 0; do
  NIDT_WGD_ADMA=$A timeout -k 10 500 python3 -u tools/config5_resnet3d.py --clients 256 --train-per-client 36 --test-per-client 9 --batch 4 --group 32 --rounds 3 --warmup 1 > $OUT/c5_$A.txt 2>&1 || { tail -20 $OUT/c5_$A.txt; exit 1; }
  echo "== WGD_ADMA=$A config5"; tail -3 $OUT/c5_$A.txt | cut -c1-300
done
