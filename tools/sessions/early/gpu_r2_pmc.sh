#!/bin/bash
# Round-2 hardware counters: the AlexNet3D hot kernels (kbench, G=64) and the CIFAR ResNet-18-GN kernels (one SubAvg
# round); counters only with --kernel-trace (no trace domains), each pass its own run; summaries only come back.
set -o pipefail
mkdir -p gpurun_out/pmc2
export PYTHONUNBUFFERED=1
export KBENCH_EVAL=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SETS=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
      "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU"
      "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
      "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum")
RE='k_conv1_fwd_pool_pipe|k_conv1_wgrad_split|k_conv_fwd_dma|k_conv_wgrad_dma'
i=0
for C in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C --kernel-include-regex "$RE" --output-format csv \
      -d /tmp/pmc_a/p$i -o run -- python3 tools/kbench.py 64 3 > gpurun_out/pmc2/a$i.log 2>&1 || exit $?
  echo "alexnet pass $i done"
done
python3 tools/pmc_summary.py /tmp/pmc_a gpurun_out/pmc2/alexnet_g64.txt > /dev/null || exit 1
rm -rf /tmp/pmc_a
RE2='k_gn_fwd|k_gn_bwd|k_conv_fwd_dma|k_conv_wgrad_dma|k_pack_wp|k_res_grad'
i=0
for C in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C --kernel-include-regex "$RE2" --output-format csv \
      -d /tmp/pmc_c/p$i -o run -- python3 tools/bench_cifar.py --algorithm subavg --rounds 1 --warmup 0 --no-eval \
      > gpurun_out/pmc2/c$i.log 2>&1 || exit $?
  echo "cifar pass $i done"
done
python3 tools/pmc_summary.py /tmp/pmc_c gpurun_out/pmc2/cifar_subavg.txt > /dev/null || exit 1
rm -rf /tmp/pmc_c
