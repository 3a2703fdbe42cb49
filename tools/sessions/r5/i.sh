#!/bin/bash
# conv1 forward wave-tile kernel: bit-exactness vs the pipe kernel, autograd tests with it forced, kbench A/B
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5i; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv1_fwd_wave_tile" > $OUT/t1.txt 2>&1 || { tail -30 $OUT/t1.txt; exit 1; }
grep -E "passed|failed" $OUT/t1.txt | tail -2
NIDT_C1_FWD=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv1_fused or alexnet_train_step" > $OUT/t2.txt 2>&1 || { tail -30 $OUT/t2.txt; exit 1; }
tail -1 $OUT/t2.txt
for V in 0 1; do
  NIDT_C1_FWD=$V timeout -k 10 200 python -u tools/kbench.py 64 > $OUT/kb64_$V.txt 2>&1 || { tail -20 $OUT/kb64_$V.txt; exit 1; }
  NIDT_C1_FWD=$V timeout -k 10 200 python -u tools/kbench.py 8 > $OUT/kb8_$V.txt 2>&1 || { tail -20 $OUT/kb8_$V.txt; exit 1; }
  echo "== NIDT_C1_FWD=$V"; grep -E "full train step|conv1_fwd|eval forward" $OUT/kb64_$V.txt $OUT/kb8_$V.txt
done
