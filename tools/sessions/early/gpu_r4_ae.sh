#!/bin/bash
# Schedule A/Bs against the defaults: [SCHED-half] on the 128-channel unpadded slab blocks (NIDT_SLAB_SCHED=2, AlexNet
# conv2 forward), [SCHED] on the 128-channel per-tap blocks (NIDT_DMA_SCHED=2, the 3D ResNet 1x1 convs of config 5)
# and on the per-tap weight-gradient kernel (NIDT_WGD_SCHED=1: AlexNet conv3-5 at 8 clients, config 5) and the three-tap
# weight-gradient kernel (NIDT_WGT_SCHED=1: AlexNet conv2-5 at 64 clients)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4ae; mkdir -p $OUT
NIDT_SLAB_SCHED=2 NIDT_DMA_SCHED=2 NIDT_WGD_SCHED=1 NIDT_WGT_SCHED=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 \
  --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_resnet3d.py > $OUT/pytest.txt 2>&1 \
  || { tail -30 $OUT/pytest.txt; exit 1; }
echo "pytest all opt-ins: $(tail -1 $OUT/pytest.txt)"
for arm in 2 1 2b 1b; do
  v=${arm%b}
  NIDT_SLAB_SCHED=$v timeout -k 10 200 python tools/kbench.py 64 10 > $OUT/kb64_s$arm.txt 2>&1 || exit 1
  echo "g64 slab_sched=$arm: $(grep 'full train' $OUT/kb64_s$arm.txt) | $(grep -E 'conv2_fwd' $OUT/kb64_s$arm.txt | tr -s ' ')"
done
for arm in 1 0 1b 0b; do
  v=${arm%b}
  NIDT_WGT_SCHED=$v timeout -k 10 200 python tools/kbench.py 64 10 > $OUT/kb64_t$arm.txt 2>&1 || exit 1
  echo "g64 wgt_sched=$arm: $(grep 'full train' $OUT/kb64_t$arm.txt) | wgrad2-5 $(grep -E 'conv[2345]_wgrad' $OUT/kb64_t$arm.txt | awk '{s+=$2} END {print s}') ms"
done
for arm in 1 0 1b 0b; do
  v=${arm%b}
  NIDT_WGD_SCHED=$v timeout -k 10 200 python tools/kbench.py 8 10 > $OUT/kb8_w$arm.txt 2>&1 || exit 1
  echo "g8 wgd_sched=$arm: $(grep 'full train' $OUT/kb8_w$arm.txt) | wgrad3-5 $(grep -E 'conv[345]_wgrad' $OUT/kb8_w$arm.txt | awk '{s+=$2} END {print s}') ms"
done
for arm in base dma2 wgd1; do
  case $arm in base) e="NIDT_DMA_SCHED=1";; dma2) e="NIDT_DMA_SCHED=2";; wgd1) e="NIDT_WGD_SCHED=1";; esac
  env $e timeout -k 10 400 python3 -u tools/config5_resnet3d.py --clients 256 --train-per-client 36 \
    --test-per-client 9 --batch 4 --group 32 --rounds 3 --warmup 1 > $OUT/config5_$arm.txt 2>&1 \
    || { tail -30 $OUT/config5_$arm.txt; exit 1; }
  echo "config5 $arm: $(grep '^{' $OUT/config5_$arm.txt | grep -o '"steady_s_per_round": [0-9.]*\|"s_round_each": [^]]*]' | tr '\n' ' ')"
done
