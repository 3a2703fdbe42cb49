#!/bin/bash
# bisect the eval-mode gradient test (conv1 slot layout); wgrad_tri asm-DMA numerics + kbench A/B; rest of the suite
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6f; mkdir -p $OUT
T=tests/test_gpu_personalized.py::test_eval_mode_gradient_matches_autograd
for cfg in "NIDT_C1_TAPORD=2" "NIDT_C1_TAPORD=0" "NIDT_C1_FWD=0" "NIDT_WGT_ADMA=0"; do
  env $cfg timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread $T > $OUT/t.txt 2>&1; rc=$?
  echo "== $cfg rc=$rc"; tail -1 $OUT/t.txt
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad" > $OUT/wg.txt 2>&1 || { tail -30 $OUT/wg.txt; exit 1; }
tail -1 $OUT/wg.txt
export KBENCH_EVAL=0
for A in 1 0; do
  NIDT_WGT_ADMA=$A timeout -k 10 200 python -u tools/kbench.py 64 > $OUT/kb64_a$A.txt 2>&1 || { tail -20 $OUT/kb64_a$A.txt; exit 1; }
  echo "== ADMA=$A"; grep -E "full train step|wgrad" $OUT/kb64_a$A.txt
done
NIDT_WGT_ADMA=1 timeout -k 10 200 python -u tools/kbench.py 8 > $OUT/kb8_a1.txt 2>&1 || { tail -20 $OUT/kb8_a1.txt; exit 1; }
echo "== ADMA=1 G=8"; grep -E "full train step|wgrad" $OUT/kb8_a1.txt
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests --deselect $T > $OUT/gpu_all.txt 2>&1; echo "suite rc=$?"
tail -5 $OUT/gpu_all.txt
