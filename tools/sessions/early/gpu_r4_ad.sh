#!/bin/bash
# [SCHED] on the 64-channel k_conv_fwd_dma blocks (NIDT_DMA_SCHED=1 default vs 0): numerics, kbench G=64 / G=8,
# headline bench, config 5 (3D ResNet, 64-channel layers on the per-tap kernel)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4ad; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py \
  tests/test_gpu_resnet2d.py tests/test_gpu_resnet3d.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
echo "pytest: $(tail -1 $OUT/pytest.txt)"
for arm in 1 0 1b 0b; do
  v=${arm%b}
  NIDT_DMA_SCHED=$v timeout -k 10 200 python tools/kbench.py 64 10 > $OUT/kb64_d$arm.txt 2>&1 || exit 1
  echo "g64 dma_sched=$arm: $(grep 'full train' $OUT/kb64_d$arm.txt) | $(grep -E 'conv[345]_(fwd|dgrad)' $OUT/kb64_d$arm.txt | awk '{s+=$2} END {print "conv3-5 fwd+dgrad", s, "ms"}')"
done
for arm in 1 0 1b 0b; do
  v=${arm%b}
  NIDT_DMA_SCHED=$v timeout -k 10 200 python tools/kbench.py 8 10 > $OUT/kb8_d$arm.txt 2>&1 || exit 1
  echo "g8 dma_sched=$arm: $(grep 'full train' $OUT/kb8_d$arm.txt) | $(grep -E 'conv[345]_(fwd|dgrad)' $OUT/kb8_d$arm.txt | awk '{s+=$2} END {print "conv3-5 fwd+dgrad", s, "ms"}')"
done
for arm in 1 0; do
  NIDT_DMA_SCHED=$arm timeout -k 10 300 python bench.py > $OUT/bench_d$arm.json 2>&1 || exit 1
  echo "bench dma_sched=$arm: $(grep -o '"value": [0-9.]*' $OUT/bench_d$arm.json)"
done
for arm in 1 0; do
  NIDT_DMA_SCHED=$arm timeout -k 10 400 python3 -u tools/config5_resnet3d.py --clients 256 --train-per-client 36 \
    --test-per-client 9 --batch 4 --group 32 --rounds 3 --warmup 1 > $OUT/config5_d$arm.txt 2>&1 \
    || { tail -30 $OUT/config5_d$arm.txt; exit 1; }
  echo "config5 dma_sched=$arm: $(grep '^{' $OUT/config5_d$arm.txt | grep -o '"steady_s_per_round": [0-9.]*\|"s_round_each": [^]]*]' | tr '\n' ' ')"
done
