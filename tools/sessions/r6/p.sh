#!/bin/bash
# wgrad1x1.hip: tests, per-layer weight-gradient timing (new kernel vs k_conv_wgrad_dma), config 5 steady rounds
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6p; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_resnet3d.py > $OUT/t.txt 2>&1 || { grep -E "PASS|FAIL|Error|assert" $OUT/t.txt | tail -30; exit 1; }
grep -E "passed|failed" $OUT/t.txt | tail -1
NIDT_WG1X1=0 timeout -k 10 300 python -u tools/bench_wgrad3d.py > $OUT/wg_old.txt 2>&1 || { tail -20 $OUT/wg_old.txt; exit 1; }
timeout -k 10 300 python -u tools/bench_wgrad3d.py > $OUT/wg_new.txt 2>&1 || { tail -20 $OUT/wg_new.txt; exit 1; }
echo "== k_conv_wgrad_dma"; grep -v amdgpu.ids $OUT/wg_old.txt
echo "== wgrad1x1"; grep -v amdgpu.ids $OUT/wg_new.txt
for v in 0 1; do
NIDT_WG1X1=$v timeout -k 10 600 python3 -u tools/config5_resnet3d.py \
  --clients 256 --train-per-client 36 --test-per-client 9 --batch 4 --group 32 --rounds 3 --warmup 1 \
  > $OUT/config5_$v.txt 2>&1 || { tail -30 $OUT/config5_$v.txt; exit 1; }
echo "== config5 NIDT_WG1X1=$v"; grep -E '^round|steady' $OUT/config5_$v.txt | cut -c1-300
done
