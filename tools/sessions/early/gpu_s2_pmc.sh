#!/bin/bash
# Hardware counters of the G=64 kbench with the session-2 kernels (union-staged wgrad/forward): two passes, counters
# only with --kernel-trace; summaries come back (tools/pmc_summary.py)
set -o pipefail
mkdir -p gpurun_out/pmc3
export PYTHONUNBUFFERED=1 KBENCH_EVAL=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SETS=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"
      "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY TCC_HIT_sum TCC_MISS_sum")
RE='k_conv1_fwd_pool_pipe|k_conv1_wgrad_split|k_conv_fwd_dma|k_conv_fwd_tri|k_conv_wgrad_tri|k_conv_wgrad_dma'
i=0
for C in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $C --kernel-include-regex "$RE" --output-format csv \
      -d /tmp/pmc3/p$i -o run -- python3 tools/kbench.py 64 3 > gpurun_out/pmc3/a$i.log 2>&1 || exit $?
  echo "pass $i done"
done
python3 tools/pmc_summary.py /tmp/pmc3 gpurun_out/pmc3/alexnet_g64.txt > /dev/null || exit 1
grep "==\|derived" gpurun_out/pmc3/alexnet_g64.txt
