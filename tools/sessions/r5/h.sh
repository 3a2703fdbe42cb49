#!/bin/bash
# (1) the 8-rank headline layout rehearsed on one GPU (gloo, 64 clients, 8 per rank) vs the 1-rank run;
# (2) kbench step times at 64 and 8 clients; (3) PMC passes over kbench 64 incl. the smfmac conv1 weight gradient
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5h; mkdir -p $OUT
timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 > $OUT/one_rank.txt 2>&1 || { tail -20 $OUT/one_rank.txt; exit 1; }
tail -1 $OUT/one_rank.txt
NIDT_DIST_BACKEND=gloo timeout -k 20 400 python -u bench.py --gpus 8 --steps 2 --warmup 1 > $OUT/eight_ranks.txt 2>&1 || { tail -30 $OUT/eight_ranks.txt; exit 1; }
grep "^{" $OUT/eight_ranks.txt
timeout -k 10 200 python -u tools/kbench.py 64 > $OUT/kbench64.txt 2>&1 || { tail -20 $OUT/kbench64.txt; exit 1; }
timeout -k 10 200 python -u tools/kbench.py 8 > $OUT/kbench8.txt 2>&1 || { tail -20 $OUT/kbench8.txt; exit 1; }
grep -i "step" $OUT/kbench64.txt $OUT/kbench8.txt | tail -6
export KBENCH_EVAL=0
RE='k_conv1_fwd_pool_pipe|k_conv1_wgrad_mx|k_conv1_wgrad_fin|k_conv_fwd_slab|k_conv_wgrad_tri|k_conv_fwd_dma|k_bn_bwd_dx|k_local_step'
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
grep -E "^==|derived" $OUT/pmc_summary.txt
