#!/bin/bash
# 64-channel slab forward / data-gradient kernel variants (the AlexNet conv2 data gradient): [SCHED] fragment
# schedule (NIDT_SLAB_SCHED=1) and 8-wave blocks (NIDT_SLAB_WM64=2) against the default; numerics first, then kbench
# G=64 / G=8 interleaved
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4ab; mkdir -p $OUT
for v in "NIDT_SLAB_SCHED=1" "NIDT_SLAB_WM64=2"; do
  env $v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
    -k "slab or alexnet or fwd" > $OUT/pytest_${v%%=*}.txt 2>&1 || { tail -30 $OUT/pytest_${v%%=*}.txt; exit 1; }
  echo "$v: $(tail -1 $OUT/pytest_${v%%=*}.txt)"
done
for arm in base sched wm2 base2 sched2 wm22; do
  case $arm in base*) e="NIDT_SLAB_SCHED=0";; sched*) e="NIDT_SLAB_SCHED=1";; wm2*) e="NIDT_SLAB_WM64=2";; esac
  env $e timeout -k 10 200 python tools/kbench.py 64 10 > $OUT/kb64_$arm.txt 2>&1 || { tail -5 $OUT/kb64_$arm.txt; exit 1; }
  echo "g64 $arm: $(grep 'full train' $OUT/kb64_$arm.txt) | $(grep -E 'conv2_(fwd|dgrad)' $OUT/kb64_$arm.txt | tr -s ' ' | tr '\n' ' ')"
done
for arm in base sched wm2; do
  case $arm in base*) e="NIDT_SLAB_SCHED=0";; sched*) e="NIDT_SLAB_SCHED=1";; wm2*) e="NIDT_SLAB_WM64=2";; esac
  env $e timeout -k 10 200 python tools/kbench.py 8 10 > $OUT/kb8_$arm.txt 2>&1 || { tail -5 $OUT/kb8_$arm.txt; exit 1; }
  echo "g8 $arm: $(grep 'full train' $OUT/kb8_$arm.txt) | $(grep -E 'conv2_(fwd|dgrad)' $OUT/kb8_$arm.txt | tr -s ' ' | tr '\n' ' ')"
done
