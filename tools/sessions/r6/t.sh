#!/bin/bash
# config 5: 3x3x3 stride-1 weight gradients on the union-staged kernels (slab / tri) + an env sweep of wgrad switches
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6t; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_resnet3d.py > $OUT/t.txt 2>&1 || { grep -E "PASS|FAIL|Error|assert" $OUT/t.txt | tail -30; exit 1; }
grep -E "passed|failed" $OUT/t.txt | tail -1
NIDT_R3D_WG_UNION=0 timeout -k 10 300 python -u tools/bench_wgrad3d.py > $OUT/wg_old.txt 2>&1 || { tail -20 $OUT/wg_old.txt; exit 1; }
timeout -k 10 300 python -u tools/bench_wgrad3d.py > $OUT/wg_new.txt 2>&1 || { tail -20 $OUT/wg_new.txt; exit 1; }
echo "== wgrad k_conv_wgrad_dma"; grep "k=3" $OUT/wg_old.txt
echo "== wgrad union"; grep "k=3" $OUT/wg_new.txt
C5="--clients 256 --train-per-client 36 --test-per-client 9 --batch 4 --group 32 --rounds 3 --warmup 1"
i=0
for cfg in "NIDT_R3D_WG_UNION=0" "X=0" "NIDT_WG_DIRECT=2" "NIDT_WGRAD_STREAM=1"; do
  i=$((i+1))
  env $cfg timeout -k 10 600 python3 -u tools/config5_resnet3d.py $C5 > $OUT/c5_$i.txt 2>&1 || { tail -30 $OUT/c5_$i.txt; exit 1; }
  echo "== $cfg $(grep -o '"steady_s_per_round": [0-9.]*' $OUT/c5_$i.txt)"; grep -E '^round' $OUT/c5_$i.txt
done
