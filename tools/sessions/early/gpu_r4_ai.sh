#!/bin/bash
# [SCHED] on every 128-channel per-tap forward block (NIDT_DMA_SCHED=2) at 8 clients (k_conv_fwd_dma<128,2,1,3>:
# AlexNet conv5 forward / conv3 data gradient) vs the default
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4ai; mkdir -p $OUT
NIDT_DMA_SCHED=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_kernels.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
echo "pytest dma_sched=2: $(tail -1 $OUT/pytest.txt)"
for arm in 2 1 2b 1b 2c 1c; do
  v=${arm%[bc]}
  NIDT_DMA_SCHED=$v timeout -k 10 200 python tools/kbench.py 8 10 > $OUT/kb8_d$arm.txt 2>&1 || exit 1
  echo "g8 dma_sched=$arm: $(grep 'full train' $OUT/kb8_d$arm.txt) | conv3-5 fwd+dgrad $(grep -E 'conv[345]_(fwd|dgrad)' $OUT/kb8_d$arm.txt | awk '{s+=$2} END {print s}') ms"
done
for arm in 2 1 2b 1b; do
  v=${arm%b}
  NIDT_DMA_SCHED=$v timeout -k 10 300 python bench.py --clients 8 --steps 30 --warmup 5 > $OUT/c8_d$arm.json 2>&1 || exit 1
  echo "c8 dma_sched=$arm: $(grep -o '"value": [0-9.]*' $OUT/c8_d$arm.json)"
done
