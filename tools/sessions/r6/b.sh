#!/bin/bash
# conv1 forward RO=2 (all-b128 k-slot layout): numerics tests, kbench G=64/G=8, LDS-conflict PMC pass
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6b; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "conv1" > $OUT/t.txt 2>&1 || { tail -30 $OUT/t.txt; exit 1; }
tail -2 $OUT/t.txt
for T in 2 0; do
  NIDT_C1_TAPORD=$T timeout -k 10 200 python -u tools/kbench.py 64 > $OUT/kb64_t$T.txt 2>&1 || { tail -20 $OUT/kb64_t$T.txt; exit 1; }
  echo "== TAPORD=$T"; grep -E "full train step|conv1_fwd|eval forward" $OUT/kb64_t$T.txt
done
timeout -k 10 200 python -u tools/kbench.py 8 > $OUT/kb8.txt 2>&1 || { tail -20 $OUT/kb8.txt; exit 1; }
grep -E "full train step|conv1_fwd" $OUT/kb8.txt
export KBENCH_EVAL=0
RE='k_conv1_fwd_w64'
i=0
for C in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C --kernel-include-regex "$RE" --output-format csv \
      -d /tmp/pmc/p$i -o run -- python3 tools/kbench.py 64 2 > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py /tmp/pmc $OUT/pmc_summary.txt > /dev/null 2>&1 || true
cat $OUT/pmc_summary.txt | cut -c1-250
