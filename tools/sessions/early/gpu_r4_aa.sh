#!/bin/bash
# AlexNet conv2-5 weight packs batched into two pack.hip launches (NIDT_AX_BPACK=1): numerics, then interleaved A/B
# at 8 clients (launch-bound) and 64 clients per GPU
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4aa; mkdir -p $OUT
NIDT_AX_BPACK=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_runner.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -k "alexnet or graph or training_log" > $OUT/pytest.txt 2>&1 \
  || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for arm in 1 0 1b 0b 1c 0c; do
  v=${arm%[bc]}
  NIDT_AX_BPACK=$v timeout -k 10 300 python bench.py --clients 8 --steps 30 --warmup 5 > $OUT/c8_b$arm.json 2>&1 || exit 1
  echo "c8 bpack=$arm: $(grep -o '"value": [0-9.]*' $OUT/c8_b$arm.json)"
done
for arm in 1 0 1b 0b; do
  v=${arm%[bc]}
  NIDT_AX_BPACK=$v timeout -k 10 300 python bench.py > $OUT/c64_b$arm.json 2>&1 || exit 1
  echo "c64 bpack=$arm: $(grep -o '"value": [0-9.]*' $OUT/c64_b$arm.json)"
done
