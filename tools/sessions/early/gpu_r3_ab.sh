#!/bin/bash
# Evidence for the round-3 kernels: PMC passes over kbench (slab forward, conv1 forward, wgrads) and a windowed
# rocprofv3 kernel timeline of one bench round
set -o pipefail
mkdir -p gpurun_out/r3ab
export PYTHONUNBUFFERED=1 KBENCH_EVAL=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
RE='k_conv1_fwd_pool_pipe|k_conv1_wgrad_split|k_conv_fwd_dma|k_conv_fwd_slab|k_conv_fwd_tri|k_conv_wgrad_tri'
i=0
for C in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
         "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C --kernel-include-regex "$RE" --output-format csv \
      -d gpurun_out/r3ab/p$i -o run -- python3 tools/kbench.py 64 3 > gpurun_out/r3ab/p$i.log 2>&1 || exit $?
  echo "pmc pass $i done"
done
python3 tools/pmc_summary.py gpurun_out/r3ab gpurun_out/r3ab/pmc_summary.txt > /dev/null 2>&1 || true
head -5 gpurun_out/r3ab/pmc_summary.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/profab -o run -- python3 -u bench.py --steps 2 --warmup 1 \
  > gpurun_out/r3ab/prof.txt 2>&1 || { tail -20 gpurun_out/r3ab/prof.txt; exit 1; }
db=$(find /tmp/profab -name "*.db" | head -1)
python3 tools/prof_summary.py --top 45 --window-ms 460 "$db" > gpurun_out/r3ab/round_kernels.txt 2>&1
head -24 gpurun_out/r3ab/round_kernels.txt; grep -E "TOTAL|TIMELINE" gpurun_out/r3ab/round_kernels.txt
