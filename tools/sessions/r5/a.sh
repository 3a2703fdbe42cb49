#!/bin/bash
# round 5: conv1 weight gradient on the argmax-row smfmac kernel (k_conv1_wgrad_mx) — numerics vs the VALU gather,
# then kbench at 64 and 8 clients (mx default) and the VALU kernel for comparison
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5a; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "conv1_wgrad_smfmac or conv1_fused" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -3 $OUT/pytest.txt
timeout -k 10 200 python -u tools/kbench.py 64 5 > $OUT/kb64_mx.txt 2>&1 || { tail -20 $OUT/kb64_mx.txt; exit 1; }
head -4 $OUT/kb64_mx.txt
NIDT_C1WG_MX=0 timeout -k 10 200 python -u tools/kbench.py 64 5 > $OUT/kb64_valu.txt 2>&1 || exit 1
head -4 $OUT/kb64_valu.txt
timeout -k 10 200 python -u tools/kbench.py 8 5 > $OUT/kb8_mx.txt 2>&1 || exit 1
head -4 $OUT/kb8_mx.txt
NIDT_C1WG_MX=0 timeout -k 10 200 python -u tools/kbench.py 8 5 > $OUT/kb8_valu.txt 2>&1 || exit 1
head -4 $OUT/kb8_valu.txt
