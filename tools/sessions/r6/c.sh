#!/bin/bash
# conv1 forward RO=2 prefetch distance A/B (kbench 64), gemm1x1 STATS drain test
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6c; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_resnet3d.py -k "gemm1x1" > $OUT/t.txt 2>&1 || { tail -30 $OUT/t.txt; exit 1; }
tail -2 $OUT/t.txt
export KBENCH_EVAL=0
for P in 2 3 4; do
  NIDT_C1_WPF=$P timeout -k 10 200 python -u tools/kbench.py 64 > $OUT/kb64_p$P.txt 2>&1 || { tail -20 $OUT/kb64_p$P.txt; exit 1; }
  echo "== WPF=$P"; grep -E "full train step|conv1_fwd" $OUT/kb64_p$P.txt
done
NIDT_C1_TAPORD=0 timeout -k 10 200 python -u tools/kbench.py 64 > $OUT/kb64_t0.txt 2>&1 || { tail -20 $OUT/kb64_t0.txt; exit 1; }
echo "== TAPORD=0"; grep -E "full train step|conv1_fwd" $OUT/kb64_t0.txt
