#!/bin/bash
# PMC record of the AlexNet3D 64-client step after the k-step schedule changes (kbench 64): MFMA busy, instruction mix, LDS
# bank conflicts, issue stalls and L2 traffic of the top kernels (summarised on the box; raw CSVs in /tmp)
set -o pipefail
export PYTHONUNBUFFERED=1 KBENCH_EVAL=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4af; mkdir -p $OUT
RE='k_conv1_fwd_pool_pipe|k_conv1_wgrad_split|k_conv_fwd_slab|k_conv_wgrad_tri|k_conv_fwd_dma|k_bn_bwd_dx|k_local_step'
i=0
for C in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
         "FETCH_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C --kernel-include-regex "$RE" --output-format csv \
      -d /tmp/pmc/p$i -o run -- python3 tools/kbench.py 64 2 > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py /tmp/pmc $OUT/pmc_summary.txt > /dev/null 2>&1 || true
grep -E "^==|derived|FETCH" $OUT/pmc_summary.txt
