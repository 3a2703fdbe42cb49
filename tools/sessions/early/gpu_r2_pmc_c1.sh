#!/bin/bash
# hardware counters of the conv1 kernels (kbench G=64): counters only with --kernel-trace, each pass its own run
set -o pipefail
mkdir -p gpurun_out/pmc3
export PYTHONUNBUFFERED=1
export KBENCH_EVAL=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SETS=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
      "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU"
      "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
      "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum")
RE='k_conv1_fwd_pool_pipe|k_conv1_wgrad_split'
i=0
for C in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C --kernel-include-regex "$RE" --output-format csv \
      -d /tmp/pmc_a/p$i -o run -- python3 tools/kbench.py 64 3 > gpurun_out/pmc3/a$i.log 2>&1 || exit $?
  echo "pass $i done"
done
python3 tools/pmc_summary.py /tmp/pmc_a gpurun_out/pmc3/conv1_g64.txt > /dev/null || exit 1
rm -rf /tmp/pmc_a
cat gpurun_out/pmc3/conv1_g64.txt | grep -E "==|derived"
