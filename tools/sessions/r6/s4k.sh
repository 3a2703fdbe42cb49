#!/bin/bash
# end-of-round evidence over the DEFAULT kernel set (after the statistics-epilogue work): 64- and 8-client round
# traces (rocprofv3 kernel-trace, timed rounds only) and PMC passes over kbench 64
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s4k; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/rt64 -o run -- python3 -u bench.py --steps 3 --warmup 2 > $OUT/b64.txt 2>&1 || { tail -20 $OUT/b64.txt; exit 1; }
tail -1 $OUT/b64.txt | cut -c1-200
db=$(find /tmp/rt64 -name "*.db" | head -1)
W=$(python3 -c "import json; d=[json.loads(l) for l in open('$OUT/b64.txt') if l.startswith('{')][-1]; print(int(d['ms_per_step']*d['steps']))")
python3 tools/prof_summary.py "$db" $OUT/c64_round_kernels.txt --top 45 --window-ms "$W" > /dev/null 2>&1 || true
head -12 $OUT/c64_round_kernels.txt | cut -c1-160
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/rt8 -o run -- python3 -u bench.py --clients 8 --steps 10 --warmup 3 > $OUT/b8.txt 2>&1 || { tail -20 $OUT/b8.txt; exit 1; }
tail -1 $OUT/b8.txt | cut -c1-200
db=$(find /tmp/rt8 -name "*.db" | head -1)
W=$(python3 -c "import json; d=[json.loads(l) for l in open('$OUT/b8.txt') if l.startswith('{')][-1]; print(int(d['ms_per_step']*d['steps']))")
python3 tools/prof_summary.py "$db" $OUT/c8_round_kernels.txt --top 45 --window-ms "$W" > /dev/null 2>&1 || true
head -12 $OUT/c8_round_kernels.txt | cut -c1-160
export KBENCH_EVAL=0
RE='k_conv1_fwd_w64|k_conv1_wgrad_mx|k_conv_fwd_slab|k_conv_wgrad_tri|k_conv_fwd_dma|k_bn_bwd_dx|k_local_step|k_bn_relu_pool'
i=0
for C in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
         "FETCH_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $C --kernel-include-regex "$RE" --output-format csv \
      -d /tmp/pmc/p$i -o run -- python3 tools/kbench.py 64 2 > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py /tmp/pmc $OUT/pmc_summary.txt > /dev/null 2>&1 || true
grep -E "^==|derived" $OUT/pmc_summary.txt | cut -c1-230
