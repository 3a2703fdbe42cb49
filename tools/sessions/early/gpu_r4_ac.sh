#!/bin/bash
# [SCHED] default for the 64-channel slab blocks: kernel + ResNet numerics, kbench G=64/G=8 and bench.py A/B
# (NIDT_SLAB_SCHED=1 default vs 0), CIFAR SubAvg A/B (2-D 64-channel slab layers)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4ac; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py \
  tests/test_gpu_resnet2d.py tests/test_gpu_resnet3d.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
echo "pytest: $(tail -1 $OUT/pytest.txt)"
for arm in 1 0 1b 0b; do
  v=${arm%b}
  NIDT_SLAB_SCHED=$v timeout -k 10 200 python tools/kbench.py 64 10 > $OUT/kb64_s$arm.txt 2>&1 || exit 1
  echo "g64 sched=$arm: $(grep 'full train' $OUT/kb64_s$arm.txt) | $(grep -E 'conv2_dgrad' $OUT/kb64_s$arm.txt | tr -s ' ')"
done
for arm in 1 0; do
  NIDT_SLAB_SCHED=$arm timeout -k 10 200 python tools/kbench.py 8 10 > $OUT/kb8_s$arm.txt 2>&1 || exit 1
  echo "g8 sched=$arm: $(grep 'full train' $OUT/kb8_s$arm.txt)"
done
for arm in 1 0 1b 0b; do
  v=${arm%b}
  NIDT_SLAB_SCHED=$v timeout -k 10 300 python bench.py > $OUT/bench_s$arm.json 2>&1 || exit 1
  echo "bench sched=$arm: $(grep -o '"value": [0-9.]*' $OUT/bench_s$arm.json)"
done
for arm in 1 0; do
  NIDT_SLAB_SCHED=$arm timeout -k 10 300 python tools/bench_cifar.py --rounds 2 > $OUT/cifar_s$arm.txt 2>&1 || exit 1
  echo "cifar subavg sched=$arm: $(grep -oE '"(rounds_per_s|s_round)[a-z_]*": [0-9.]*' $OUT/cifar_s$arm.txt | tr '\n' ' ')"
done
