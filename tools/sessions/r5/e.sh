#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5h; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "conv1_wgrad_smfmac or conv1_fused" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
for arm in 0 1; do
  NIDT_C1WG_DBG=$arm timeout -k 10 200 python -u tools/kbench.py 64 5 > $OUT/kb64_dbg$arm.txt 2>&1 || exit 1
  echo "dbg=$arm $(grep conv1_wgrad $OUT/kb64_dbg$arm.txt)"
done
timeout -k 10 200 python -u tools/kbench.py 8 5 > $OUT/kb8.txt 2>&1 || exit 1
grep "conv1_wgrad\|step" $OUT/kb8.txt
